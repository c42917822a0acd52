#!/bin/bash
# Round 6: the learner's column sums on a forked stream beside the weight gradients (MUZ_COLSUM_SIDE) on / off;
# det / DOG steps (2 reps), a det trace, the learner GPU tests.
set -o pipefail
O=gpurun_out/r6ac
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for game in det dog; do
    for cs in 0 1; do
      echo "== $game colsum_side $cs" >> $O/steps.log
      MUZ_COLSUM_SIDE=$cs timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game 2>&1 | grep "ms per step" >> $O/steps.log || exit 1
    done
  done
done
cat $O/steps.log
bash profiles/r5_learner_trace.sh r6ac_det det || exit 1
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo r6ac-done
