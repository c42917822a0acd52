#!/bin/bash
# Round 6: root inference with the paired conv workgroups at 4 waves (libmuz_convpair1) and 8 waves (the build) against
# one game per workgroup (libmuz_convpair0); the learner step with the fused GEMM + LayerNorm forward for the narrow
# layers (MUZ_FUSED_FWD_NARROW) on / off; then the learner and root-path GPU tests on the build.
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
export TMPDIR=/tmp
V=exploring-muzero-on-dog_amd/variants
NEW=exploring-muzero-on-dog_amd/libmuz.so
for rep in 1 2 3; do
  for lib in $V/libmuz_convpair0.so $V/libmuz_convpair1.so $NEW; do
    MUZ_LIB=$lib timeout -k 10 120 python3 profiles/root_microbench.py 4096 2>&1 | grep root_inference >> $O/root_ab.log || exit 1
  done
done
cat $O/root_ab.log
for rep in 1 2; do
  for game in det dog; do
    for nar in 0 1; do
      echo "== $game narrow $nar" >> $O/steps.log
      MUZ_FUSED_FWD_NARROW=$nar timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game >> $O/steps.log 2>&1 || { tail -20 $O/steps.log; exit 1; }
    done
  done
done
grep -v "^/opt\|amdgpu.ids\|selects" $O/steps.log
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_nets.py tests/test_gpu_dog_muzero.py \
  tests/test_gpu_selfplay.py tests/test_gpu_stochastic.py tests/test_gpu_headline.py tests/test_gpu_selfplay_classic.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo r6o-done
