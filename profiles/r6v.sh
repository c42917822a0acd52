#!/bin/bash
# Round 6: one weight-packing launch per learner step (up to 32 matrices), and 128-row weight-gradient segments as a
# variant; det / DOG learner steps, a det step trace, the learner GPU tests.
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
export TMPDIR=/tmp
V=exploring-muzero-on-dog_amd/variants
NEW=exploring-muzero-on-dog_amd/libmuz.so
for rep in 1 2; do
  for game in det dog; do
    for lib in $NEW $V/libmuz_wseg128.so; do
      echo "== $game $(basename $lib)" >> $O/steps.log
      MUZ_LIB=$lib timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game 2>&1 | grep "ms per step" >> $O/steps.log || exit 1
    done
  done
done
cat $O/steps.log
bash profiles/r5_learner_trace.sh r6v_det det || exit 1
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo r6v-done
