#!/bin/bash
# Round 5: one weight-packing launch per learner step (learner.prepack: the representation / prediction ResBlock stacks
# and the trunk chain from one muz_trunk_chain_pack) -- learner GPU tests, det / DOG step times, det step trace.
set -o pipefail
O=gpurun_out/${R5ZG_OUT:-r5zg}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 200 python3 profiles/r5_learner_steps.py 30 det > $O/steps_$rep.log 2>&1 || { tail $O/steps_$rep.log; exit 1; }
  grep 'ms per step' $O/steps_$rep.log
done
timeout -k 10 200 python3 profiles/r5_learner_steps.py 30 dog > $O/steps_dog.log 2>&1 || { tail $O/steps_dog.log; exit 1; }
grep 'ms per step' $O/steps_dog.log
bash profiles/r5_learner_trace.sh ${R5ZG_OUT:-r5zg} det > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
head -1 gpurun_out/prof_learner_${R5ZG_OUT:-r5zg}/step_per_kernel.txt
