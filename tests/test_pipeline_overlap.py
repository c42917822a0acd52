"""pipeline.run_overlapped (config (e)'s overlapped actor / learner iterations) on CPU: with gloo over 3 ranks
(2 actors + 1 learner) and in one process with the actor in a thread.  Every game reaches the learner's ring
exactly once, and generation g is played with the weights of iteration g - 2 -- exactly one iteration staler
than the reference's sequential loop (train_with_reward.py:244-292), where it would be g - 1."""
import os
import socket
import threading

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

GAMES_PER_ACTOR = 3
ITERS = 5


def _pl():
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import pipeline
    return pipeline


def _check_ring(ring, actors):
    ids = [int(r[0]) for r in ring]
    assert len(ids) == len(set(ids)) == (ITERS + 1) * GAMES_PER_ACTOR * actors, "a game missing or duplicated"
    for gid, gen, ver in ring:
        want = -1 if gen <= 1 else gen - 2          # sequential: gen - 1 (W_-1 = initial weights)
        assert int(ver) == want, (int(gid), int(gen), int(ver))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P = _pl()
    learner = world - 1
    net = {"w": torch.tensor([-1.0])}          # the weights an actor holds (version number)
    version = {"v": -1}                        # the learner's newest weights
    ring, trained_on = [], []

    def play(g):
        base = (g * (world - 1) + rank) * GAMES_PER_ACTOR
        return torch.tensor([[base + j, g, float(net["w"])] for j in range(GAMES_PER_ACTOR)])

    def train(i):
        trained_on.append((i, max(int(r[1]) for r in ring)))
        version["v"] = i

    def deliver(g, games):
        mine = games if games is not None else torch.zeros((GAMES_PER_ACTOR, 3))
        out = [torch.zeros_like(mine) for _ in range(world)] if rank == learner else None
        dist.gather(mine, out, dst=learner)
        if rank == learner:
            for r in range(world - 1):
                ring.extend(out[r].tolist())

    class _H:
        def __init__(self, work, buf):
            self.work, self.buf = work, buf

        def wait(self):
            self.work.wait()
            if rank != learner:
                net["w"] = self.buf.clone()

    def publish(i):
        buf = torch.tensor([float(version["v"])]) if rank == learner else torch.zeros(1)
        return _H(dist.broadcast(buf, src=learner, async_op=True), buf)

    n = P.run_overlapped(ITERS, is_actor=rank != learner, is_learner=rank == learner, play=play, train=train,
                         deliver=deliver, publish=publish)
    res = None
    if rank == learner:
        _check_ring(ring, world - 1)
        # iteration i trains on generations 0..i (generation i+1 is still being played)
        assert all(last == i for i, last in trained_on), trained_on
        res = n
    q.put((rank, res))
    dist.destroy_process_group()


def test_overlap_three_ranks_gloo():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[world - 1] == ITERS + 1


def test_overlap_one_process_threads():
    """Both roles in one process (one GPU): generation i+1 is played in a worker thread WHILE iteration i trains
    (the two calls overlap in time), weights pushed at the barrier."""
    P = _pl()
    net = {"w": -1}
    ring, trained = [], {"v": -1}
    overlap = {"n": 0}
    in_train = threading.Event()

    def play(g):
        if g > 0:                                 # generation g > 0 is played while train(g - 1) runs
            overlap["n"] += int(in_train.wait(timeout=10))
        return [(g * GAMES_PER_ACTOR + j, g, net["w"]) for j in range(GAMES_PER_ACTOR)]

    def train(i):
        in_train.set()
        import time
        time.sleep(0.01)
        in_train.clear()
        trained["v"] = i

    class _Push:
        def wait(self):
            pass

    def publish(i):
        net["w"] = trained["v"]
        return _Push()

    n = P.run_overlapped(ITERS, is_actor=True, is_learner=True, play=play, train=train,
                         deliver=lambda g, games: ring.extend(games), publish=publish, concurrent=True)
    assert n == ITERS + 1 and overlap["n"] == ITERS
    _check_ring(ring, 1)


def test_weight_update_wait_applies_and_orders():
    """transfer._WeightUpdate.wait: completes the broadcast, rebuilds the receiver's derived
    tables once, and is idempotent; the sender does not rebuild.  (On the GPU it also synchronises the current
    stream, so self-play / learner streams cannot race the arena; a CPU buffer skips that.)"""
    import muzpkg
    muzpkg.load()
    from exploring_muzero_on_dog_amd import transfer as TR

    class Work:
        def __init__(self):
            self.waited = 0

        def wait(self):
            self.waited += 1

    class Net:
        def __init__(self):
            self.buffer = torch.zeros(8)
            self.prepared = 0

        def prepare(self):
            self.prepared += 1

    for receiver in (True, False):
        w, net = Work(), Net()
        h = TR._WeightUpdate(w, net, receiver)
        h.wait()
        h.wait()
        assert w.waited == 1
        assert net.prepared == (1 if receiver else 0)
