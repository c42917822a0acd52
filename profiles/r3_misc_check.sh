#!/bin/bash
# (1) the driver's multi-GPU launch path on the one-GPU box: torchrun with one rank over RCCL (nccl backend),
# (2) kernel-trace summary of the classic (config c) bench, one step.
set -o pipefail
O=gpurun_out/r3_misc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --steps 1 --warmup 1 --no-cpu-baseline > $O/torchrun_n1.json 2> $O/torchrun_n1.err || { tail -20 $O/torchrun_n1.err; exit 1; }
tail -1 $O/torchrun_n1.json | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/classic_trace -o run --output-format csv -- \
  python3 bench.py --workload classic --steps 1 --warmup 1 --no-cpu-baseline > $O/classic_trace.log 2>&1 || { tail -20 $O/classic_trace.log; exit 1; }
find $O -name '*_kernel_trace.csv' -delete
f=$(find $O/classic_trace -name 'run_kernel_stats.csv' | head -1)
head -14 "$f" | cut -d, -f1-5
