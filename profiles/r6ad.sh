#!/bin/bash
# Round 6: the AdamW update with 16-byte accesses (k_adam_update_t) against the scalar form (libmuz_adam0): det / DOG
# learner steps, the trained parameters compared bit for bit, a det trace, the learner GPU tests.
set -o pipefail
O=gpurun_out/r6ad
mkdir -p $O
export TMPDIR=/tmp
OLD=exploring-muzero-on-dog_amd/variants/libmuz_adam0.so
NEW=exploring-muzero-on-dog_amd/libmuz.so
for game in det dog; do
  for tag in old new; do
    lib=$OLD; [ $tag = new ] && lib=$NEW
    echo "== $game $tag" >> $O/steps.log
    MUZ_LIB=$lib MUZ_DUMP=$O/${game}_$tag.npz timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game 2>&1 | grep "ms per step" >> $O/steps.log || exit 1
  done
done
for tag in old new; do
  lib=$OLD; [ $tag = new ] && lib=$NEW
  echo "== det $tag (rep 2)" >> $O/steps.log
  MUZ_LIB=$lib timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 det 2>&1 | grep "ms per step" >> $O/steps.log || exit 1
done
cat $O/steps.log
python3 - <<'PY' | tee $O/bitcheck.log
import numpy as np
for g in ("det", "dog"):
    a, b = np.load(f"gpurun_out/r6ad/{g}_old.npz"), np.load(f"gpurun_out/r6ad/{g}_new.npz")
    diff = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
    print(f"{g}: {len(a.files)} parameters after 63 steps, {len(diff)} differ bitwise", diff[:8])
PY
bash profiles/r5_learner_trace.sh r6ad_det det || exit 1
grep adam gpurun_out/prof_learner_r6ad_det/step_per_kernel.txt
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo r6ad-done
