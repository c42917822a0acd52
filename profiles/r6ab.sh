#!/bin/bash
# Round 6: the N-rank bench path rehearsed on one GPU (2 ranks sharing it, gloo collectives: MUZ_BENCH_BACKEND=gloo_gpu)
# -- bench.py's own launcher and torch.distributed.run, the barrier / max-over-ranks timing and rank 0's line.
set -o pipefail
O=gpurun_out/r6ab
mkdir -p $O
export TMPDIR=/tmp
export MUZ_BENCH_BACKEND=gloo_gpu
timeout -k 10 500 python3 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > $O/self_launch.json 2> $O/self_launch.err || { tail -20 $O/self_launch.err; exit 1; }
tail -1 $O/self_launch.json | cut -c1-400
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > $O/torchrun.json 2> $O/torchrun.err || { tail -20 $O/torchrun.err; exit 1; }
tail -1 $O/torchrun.json | cut -c1-400
echo r6ab-done
