#!/bin/bash
# Round 6: unit tests of the round's learner launch forms (strided-gradient backward, split-K LayerNorm epilogue,
# segment sums), bit for bit against the forms they replace.
set -o pipefail
O=gpurun_out/r6af
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_learner_strided.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -12
echo r6af-done
