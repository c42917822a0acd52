#!/bin/bash
# Round 5 final: the headline bench line (default flags) and its rocprofv3 kernel statistics on HEAD.
set -o pipefail
O=gpurun_out/r5zq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name '*_kernel_trace.csv' -delete
head -3 $O/kernel_stats.csv | cut -c1-100
