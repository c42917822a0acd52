"""The multi-rank path of bench.py (sum of work, max of time over ranks) on CPU with gloo, world_size 2."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    sums, elapsed = bench.sum_max(dist, torch.device("cpu"), [100 * (rank + 1), 10 * (rank + 1), 5.0, 3],
                                  elapsed=1.0 + rank)
    res = (sums[0], sums[1], elapsed, sums[2], sums[3])
    q.put((rank, res))
    dist.destroy_process_group()


def test_bench_reduction_two_ranks():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        steps, searches, elapsed, search_ms, launches = out[r]
        assert steps == 300 and searches == 30 and elapsed == 2.0 and search_ms == 10.0 and launches == 6


# ---- trajectory gather (actors -> learner) and weight broadcast, gloo on CPU --------------------------
def _synthetic_packed(rank, C=6, A=5, chance=False):
    """Deterministic packed games of one actor rank (what transfer.pack produces on a GPU)."""
    g = torch.Generator().manual_seed(100 + rank)
    n = 3 + rank
    idx = torch.randint(0, 9, (n,), generator=g, dtype=torch.int32)
    idx[0] = 0                                                     # a zero-length game
    off = torch.cumsum(idx.to(torch.int64), 0) - idx.to(torch.int64)
    R = int(idx.sum())
    out = {"idx": idx, "row_offset": off}
    for name, dt, shp in _fields(C, A, chance):
        if dt.is_floating_point:
            out[name] = torch.randn((R,) + shp, generator=g).to(dt)
        else:
            out[name] = torch.randint(-3, 100, (R,) + shp, generator=g, dtype=torch.int64).to(dt)
    return out


def _fields(C, A, chance):
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import transfer as T
    return T.fields(C, A, chance)


class _FakeNet:
    def __init__(self, rank):
        self.buffer = torch.full((1000,), float(rank))
        self.prepared = 0

    def prepare(self):
        self.prepared += 1


def _gather_worker(rank, world, port, q, dst, chance):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import transfer as T
    got = T.gather_packed(_synthetic_packed(rank, chance=chance), 6, 5, chance=chance, dst=dst)
    ok = True
    if rank == dst:
        ok = len(got) == world
        for r in range(world):
            want = _synthetic_packed(r, chance=chance)
            ok &= set(got[r]) == set(want) and all(torch.equal(got[r][k], want[k]) for k in want)
    else:
        ok = got is None
    net = _FakeNet(rank)
    T.broadcast_weights(net, src=dst)
    ok &= bool((net.buffer == float(dst)).all()) and net.prepared == 1
    q.put((rank, ok))
    dist.destroy_process_group()


def _run(world, dst, chance):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q, dst, chance)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(out[r] for r in range(world)), out


def test_gather_packed_two_ranks():
    _run(2, dst=0, chance=False)


def test_gather_packed_three_ranks_learner_last_with_dice():
    _run(3, dst=2, chance=True)


# ---- DOG actor records (config (d): 1024 games per GPU actor, records gathered to one learner rank) ------
def _dog_packed(rank):
    """Packed DOG records of one actor rank, built through DogTrajectory.pack on CPU tensors."""
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import dog as D
    g = torch.Generator().manual_seed(7 + rank)
    tr = D.DogTrajectory(4 + rank, 12, device="cpu")
    for k, _ in D.DOG_TRAJ_FIELDS:
        tr.buf[k].copy_(torch.randint(-1, 50, tr.buf[k].shape, generator=g).to(tr.buf[k].dtype))
    tr.buf["idx"].copy_(torch.randint(0, 13, (tr.batch,), generator=g, dtype=torch.int32))
    return tr.pack(), tr


def _dog_gather_worker(rank, world, port, q, dst):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import transfer as T
    packed, _ = _dog_packed(rank)
    got = T.gather_packed(packed, dst=dst, spec=T.dog_fields())
    ok = True
    if rank == dst:
        ok = len(got) == world
        for r in range(world):
            want, tr = _dog_packed(r)
            ok &= all(torch.equal(got[r][k], want[k]) for k in want)
            # row_offset / idx locate every game's rows: they equal the lane's record prefix
            for b in range(tr.batch):
                o, n = int(got[r]["row_offset"][b]), int(got[r]["idx"][b])
                ok &= torch.equal(got[r]["act"][o:o + n], tr.buf["act"][b, :n])
    else:
        ok = got is None
    q.put((rank, ok))
    dist.destroy_process_group()


def test_dog_records_gather_three_ranks():
    world, dst = 3, 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dog_gather_worker, args=(r, world, port, q, dst)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(out[r] for r in range(world)), out
