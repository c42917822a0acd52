#!/bin/bash
# Round-3 check of HEAD (hardware row-op reciprocals) on a fresh box: full GPU suite, smoke(), then the headline profile (bench line, kernel-trace
# summary, PMC HBM traffic of k_gumbel_search: profiles/profile_bench.sh).
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash profiles/profile_bench.sh r3h || exit 1
find gpurun_out/prof_r3h -name '*_kernel_trace.csv' -delete
