#!/bin/bash
# Kernel-trace profiles of the config (c) and (d) workloads on one MI355X (run through gpurun from the
# repo root).  Each bench runs twice: plain (-> bench json line) and under rocprofv3 --kernel-trace --stats.
# profiles/summarize_workloads.py then writes profiles/<tag>_<workload>_{bench.json,kernel_stats.csv}.
set -o pipefail
TAG=${1:-r1}
export TMPDIR=/tmp
for W in classic dog; do
  O=gpurun_out/prof_${TAG}_$W
  mkdir -p $O
  if [ $W = classic ]; then ARGS="--steps 1 --warmup 1"; else ARGS="--steps 200 --warmup 5"; fi
  timeout -k 10 300 python3 bench.py --workload $W $ARGS > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -1 $O/bench.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 bench.py --workload $W $ARGS --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
done
echo profile-done
