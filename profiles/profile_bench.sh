#!/bin/bash
# Round profile of the headline bench on one MI355X (run through gpurun from the repo root):
#   1. bench.py (default flags)                     -> $O/bench.json
#   2. rocprofv3 --kernel-trace --stats, same bench  -> $O/trace/run_kernel_stats.csv
#   3. two PMC passes (FETCH_SIZE, WRITE_SIZE) on k_gumbel_search -> $O/pmc_fetch, $O/pmc_write
# then profiles/summarize_profile.py turns them into profiles/<tag>_*.{csv,json,txt}.
set -o pipefail
TAG=${1:-r1}
O=gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_gumbel_search -d $O/pmc_fetch -o run \
  --output-format csv -- python3 bench.py --steps 1 --warmup 0 --games 8192 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_gumbel_search -d $O/pmc_write -o run \
  --output-format csv -- python3 bench.py --steps 1 --warmup 0 --games 8192 --no-cpu-baseline > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
echo profile-done
