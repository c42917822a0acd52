#!/bin/bash
# Round 5: the FiLM sub-graph (_Film, csrc/learner_film.hip) and Pred4's LayerNorm_0 (_LN) as one
# launch each way -- learner GPU tests, then the step trace.
set -o pipefail
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner_fused.py tests/test_gpu_learner.py tests/test_gpu_learner_oracle.py \
  tests/test_gpu_train_entry.py -x -v --timeout 300 --timeout-method thread > $O/learner_tests.log 2>&1 || { tail -60 $O/learner_tests.log; exit 1; }
grep -E "passed|failed|fused film|worst" $O/learner_tests.log | tail -12
bash profiles/r5_learner_trace.sh r5n det || exit 1
head -30 gpurun_out/prof_learner_r5n/step_per_kernel.txt
