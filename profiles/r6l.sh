#!/bin/bash
# Round 6 (learner <= 1.5 ms): the chain / ResBlock-stack kernels with their per-layer vectors in
# LDS and the backward's saved values loaded a layer ahead, against the round-6 head (variants/libmuz_r6chain0.so):
# chain kernels alone, the det / DOG learner step (HIP events), the trained parameters compared bit for bit, and the
# learner GPU tests on the new build.
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp
OLD=exploring-muzero-on-dog_amd/variants/libmuz_r6chain0.so
NEW=exploring-muzero-on-dog_amd/libmuz.so
for rep in 1 2; do
  for lib in $OLD $NEW; do
    echo "== $lib" >> $O/chain_bench.log
    MUZ_LIB=$lib timeout -k 10 180 python3 profiles/chain_bench.py 128 10 20 >> $O/chain_bench.log 2>&1 || { tail -20 $O/chain_bench.log; exit 1; }
  done
done
cat $O/chain_bench.log
for game in det dog; do
  for tag in old new; do
    lib=$OLD; [ $tag = new ] && lib=$NEW
    echo "== $game $tag" >> $O/steps.log
    MUZ_LIB=$lib MUZ_DUMP=$O/${game}_$tag.npz timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game >> $O/steps.log 2>&1 || { tail -20 $O/steps.log; exit 1; }
  done
done
grep -v "^/opt\|amdgpu.ids" $O/steps.log
python3 - <<'PY' | tee $O/bitcheck.log
import numpy as np
for g in ("det", "dog"):
    a, b = np.load(f"gpurun_out/r6l/{g}_old.npz"), np.load(f"gpurun_out/r6l/{g}_new.npz")
    diff = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
    print(f"{g}: {len(a.files)} parameters after 33 steps, {len(diff)} differ bitwise", diff[:8])
PY
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo r6l-done
