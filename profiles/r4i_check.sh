#!/bin/bash
# Round 4 re-entry: HEAD (ResBlock stack kernels) on a fresh MI355X -- full GPU suite, smoke, learner profile, headline.
set -o pipefail
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 800 python -u -m pytest ${TESTS:-tests} -m gpu -v --maxfail=3 --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 profiles/learner_profile.py 50 > $O/learner_profile.log 2>&1 || { tail -20 $O/learner_profile.log; exit 1; }
grep "ms$" $O/learner_profile.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
