#!/bin/bash
# Round 4: the learner's output heads as one launch each way (csrc/learner_heads.hip) -- learner GPU tests + profile.
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_learner_fused.py tests/test_gpu_learner.py tests/test_gpu_learner_oracle.py \
  tests/test_gpu_train_entry.py -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log; grep "fused heads" $O/tests.log
timeout -k 10 400 python3 profiles/learner_profile.py 50 > $O/learner_profile.log 2>&1 || { tail -20 $O/learner_profile.log; exit 1; }
grep "ms$" $O/learner_profile.log
