#!/bin/bash
# Round 5 end: rocprofv3 kernel statistics of the DOG random-policy bench (k_dog_play) and the classic bench on HEAD.
set -o pipefail
O=gpurun_out/r5zp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dog -o run --output-format csv -- python3 bench.py --workload dog --steps 2 --warmup 1 --no-cpu-baseline > $O/dog.json 2> $O/dog.err || { tail -20 $O/dog.err; exit 1; }
find $O/dog -name '*kernel_stats.csv' -exec cp {} $O/dog_kernel_stats.csv \;
find $O/dog -name '*_kernel_trace.csv' -delete
head -3 $O/dog_kernel_stats.csv | cut -c1-140
