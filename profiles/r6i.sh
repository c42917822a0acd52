#!/bin/bash
# Round 6: the headline bench line (default flags) and the rocprofv3 kernel-trace summary of the same bench command
# (k_gumbel_search's average duration must agree with the line's HIP-event avg_launch_ms); then the DOG stamp shares
# at 1500 and 256 games (profiles/r6h.sh).
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-600
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/trace -name '*_kernel_trace.csv' -delete
head -8 $O/kernel_stats.csv | cut -c1-160
tail -1 $O/trace.log | cut -c1-300
bash profiles/r6h.sh
