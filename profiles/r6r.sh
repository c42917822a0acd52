#!/bin/bash
# Round 6 (learner <= 1.5 ms): the representation's Dense_0 (K = 3584) as a batched split-K GEMM + the partial-sum
# LayerNorm (MUZ_SPLITK_DENSE) on / off, and the pipelined segment sum; det / DOG learner steps, a det step trace, the
# learner GPU tests.
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for game in det dog; do
    for sk in 0 1; do
      echo "== $game splitk $sk" >> $O/steps.log
      MUZ_SPLITK_DENSE=$sk timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game >> $O/steps.log 2>&1 || { tail -20 $O/steps.log; exit 1; }
    done
  done
done
grep -v "^/opt\|amdgpu.ids\|selects" $O/steps.log
bash profiles/r5_learner_trace.sh r6r_det det || exit 1
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo r6r-done
