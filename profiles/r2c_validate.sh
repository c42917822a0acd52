#!/bin/bash
# Re-entry check of HEAD on a fresh box: full GPU suite, smoke(), headline bench.
set -o pipefail
O=gpurun_out/${R2C_OUT:-r2c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > $O/det.json 2> $O/det.err || { tail -20 $O/det.err; exit 1; }
cat $O/det.json
