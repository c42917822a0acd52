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
    res = bench.reduce_results(dist, torch.device("cpu"), steps_done=100 * (rank + 1), searches=10 * (rank + 1),
                               elapsed=1.0 + rank, search_ms=5.0, launches=3)
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
