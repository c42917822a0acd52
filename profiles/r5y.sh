#!/bin/bash
# Round 5: (1) the fused det turn head (profiles/r5x.sh: tests + headline A/B + kernel trace), (2) the learner's
# grouped gradient launches on a side stream (ASYNC_GRADS): learner GPU tests, step-time A/B, step trace.
set -o pipefail
R5X_OUT=${R5X_OUT:-r5x2} bash profiles/r5x.sh || exit 1
[ -n "$ONLY_HEAD" ] && exit 0
O=gpurun_out/r5y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py -q --timeout 300 --timeout-method thread > $O/learner_tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/learner_tests.log | head -20; tail -3 $O/learner_tests.log; exit 1; }
tail -1 $O/learner_tests.log
for rep in 1 2; do
  for a in 0 1; do
    MUZ_ASYNC_GRADS=$a timeout -k 10 200 python3 profiles/r5_learner_steps.py 30 det > $O/steps_a${a}_${rep}.log 2>&1 || { tail $O/steps_a${a}_${rep}.log; exit 1; }
    echo "async=$a $(grep 'ms per step' $O/steps_a${a}_${rep}.log)"
  done
done
bash profiles/r5_learner_trace.sh r5y det > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
head -3 gpurun_out/prof_learner_r5y/step_per_kernel.txt
