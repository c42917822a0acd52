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


# ---- config (e) as BASELINE names it: 7 actors + 1 learner, MuZero_DOG (C = 34, A = 806) -----------------------
# bench.py run_train's two exchanges per iteration, transfer.deliver_to_learner / publish_weights, driven with the
# DOG record rows (obs int8 [34, 56], pol f32 [806]) of 2 actor ranks into the learner rank's ring (rank 2).
DOG_C, DOG_A, DOG_T = 34, 806, 24


def _dog_actor_buffers(rank):
    """[n, T] buffer dict of one DOG actor's iteration (what game_agent_dog.play_stream records), a zero-length
    game and a full-length one included; rows past idx as the reference initialises them."""
    import numpy as np
    rng = np.random.default_rng(31 + rank)
    n = 3 + 2 * rank
    idx = rng.integers(1, DOG_T, n).astype(np.int32)
    idx[0], idx[-1] = 0, DOG_T
    b = {"obs": rng.integers(0, 5, (n, DOG_T, DOG_C, 56)).astype(np.int8),
         "act": rng.integers(0, DOG_A, (n, DOG_T)).astype(np.int32),
         "rew": rng.integers(0, 3, (n, DOG_T)).astype(np.int32),
         "val": rng.standard_normal((n, DOG_T)).astype(np.float32),
         "pol": rng.dirichlet(np.ones(DOG_A), (n, DOG_T)).astype(np.float32),
         "mask": (rng.random((n, DOG_T)) > 0.1).astype(np.float32),
         "player": rng.integers(0, 4, (n, DOG_T)).astype(np.int32),
         "discount": rng.integers(0, 3, (n, DOG_T)).astype(np.int32), "idx": idx}
    b["team"] = b["player"] % 2
    for k, v in b.items():
        if k != "idx":
            v[np.arange(DOG_T)[None, :] >= idx[:, None]] = -1 if k == "team" else 0
    return b


def _host_pack_np(b):
    """transfer.pack's row layout on the host: rows [0, idx) of every game in game order (+ idx, row_offset)."""
    import numpy as np
    lens = b["idx"]
    out = {k: torch.from_numpy(np.concatenate([b[k][g, :lens[g]] for g in range(len(lens))]))
           for k in b if k != "idx"}
    out["idx"] = torch.from_numpy(lens.copy())
    out["row_offset"] = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64))
    return out


class _OracleRingPacked:
    """The learner's ring for the CPU test: oracle/replay.py's VectorizedReplayBuffer (the reference's ring restated)
    with save_packed = unpack the rows into [n, T] buffers, then save_games_from_buffers (what muz_ring_save_packed is
    tested to equal on the GPU, tests/test_gpu_replay.py)."""
    device = torch.device("cpu")

    def __init__(self, seed):
        import numpy as np
        from oracle import replay as OR
        self.ring = OR.VectorizedReplayBuffer(16, 8, 5, 10, obs_shape=(DOG_C, 56), action_dim=DOG_A,
                                              max_episode_length=DOG_T, rng=np.random.RandomState(seed))
        self.games = []

    def save_packed(self, p):
        import numpy as np
        n = p["idx"].shape[0]
        b = {}
        for name, dt, shp in _fields(DOG_C, DOG_A, False):
            v = p[name].numpy()
            buf = np.zeros((n, DOG_T) + tuple(shp), dtype=v.dtype)
            for g in range(n):
                o, L = int(p["row_offset"][g]), int(p["idx"][g])
                buf[g, :L] = v[o:o + L]
            b[name] = buf
        b["idx"] = p["idx"].numpy()
        self.games.append(n)
        self.ring.save_games_from_buffers(b)


class _FakeLearner:
    def __init__(self, value):
        self.value = value

    def push_to(self, net):
        net.buffer.fill_(self.value)


def _dog_train_worker(rank, world, port, q, learner_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import numpy as np
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import transfer as T
    from oracle import replay as OR
    ok = True
    is_learner = rank == learner_rank
    ring = _OracleRingPacked(seed=11) if is_learner else None
    packed = None if is_learner else _host_pack_np(_dog_actor_buffers(rank))
    n = T.deliver_to_learner(packed, ring, DOG_C, DOG_A, learner_rank)
    if is_learner:
        actors = [r for r in range(world) if r != learner_rank]
        ok &= n == sum(_dog_actor_buffers(r)["idx"].shape[0] for r in actors) and ring.games == [3, 5]
        # the same ring fed the actors' buffers directly, in rank order (vec_replay_buffer.py:36-61)
        want = OR.VectorizedReplayBuffer(16, 8, 5, 10, obs_shape=(DOG_C, 56), action_dim=DOG_A,
                                         max_episode_length=DOG_T, rng=np.random.RandomState(11))
        for r in actors:
            want.save_games_from_buffers(_dog_actor_buffers(r))
        got = ring.ring
        ok &= (got.position, got.size) == (want.position, want.size) == (6, 6)
        for k in ("observations", "actions", "rewards", "root_values", "child_visits", "masks", "players", "teams",
                  "discounts", "episode_lengths"):
            ok &= np.array_equal(getattr(got, k), getattr(want, k))
        bg, bw = got.sample_batch(), want.sample_batch()       # same seeded draws -> the same batch, bit for bit
        ok &= set(bg) == set(bw) and all(np.array_equal(np.asarray(bg[k]), np.asarray(bw[k])) for k in bw)
    else:
        ok &= n == 0
    net = _FakeNet(rank)
    T.publish_weights(net, _FakeLearner(float(40 + learner_rank)) if is_learner else None, learner_rank)
    ok &= bool((net.buffer == float(40 + learner_rank)).all()) and net.prepared == 1
    h = T.publish_weights(net, _FakeLearner(7.0) if is_learner else None, learner_rank, async_op=True)
    h.wait()
    ok &= bool((net.buffer == 7.0).all()) and net.prepared == (1 if is_learner else 2)
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_dog_train_exchanges_three_ranks():
    """Config (e) at A = 806: 2 actor ranks deliver their packed DOG records to the learner (rank 2, the last, as
    bench.py places it); the learner's ring and a seeded sample_batch equal the ring fed the buffers directly; then
    the learner's weights reach every rank (blocking and asynchronous broadcast)."""
    world, learner_rank = 3, 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dog_train_worker, args=(r, world, port, q, learner_rank)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(out[r] for r in range(world)), out
