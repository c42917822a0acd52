#!/bin/bash
# Round 5 final, part A: the full GPU suite, smoke, the headline bench line (default flags) and its rocprofv3 kernel
# statistics (--steps 2 --warmup 1).
set -o pipefail
O=gpurun_out/${R5F_OUT:-r5f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name '*_kernel_trace.csv' -delete
head -6 $O/kernel_stats.csv | cut -c1-120
