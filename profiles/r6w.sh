#!/bin/bash
# Round 6: the learner's loss row as a view of the fused loss kernel's parts (no stack launch in the graph), and the
# step without the loss handout copy (the bench's loop); det / DOG steps, a det trace, the learner GPU tests.
set -o pipefail
O=gpurun_out/r6w
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for game in det dog; do
    timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game 2>&1 | grep "ms per step" >> $O/steps.log || exit 1
  done
done
cat $O/steps.log
bash profiles/r5_learner_trace.sh r6w_det det || exit 1
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo r6w-done
