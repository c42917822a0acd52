#!/bin/bash
# Round 6 (learner <= 1.5 ms): k_wgrad_grouped segment length (rows per workgroup) with the per-element segment sum
# (k_seg_sum): 256 / 512 (the build) / 1024 / 2048 at the det and DOG learner step; root conv kernel traces for one game
# per workgroup, pairs on 4 waves, pairs on 8 waves (the build); the learner and root-path GPU tests.
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
export TMPDIR=/tmp
V=exploring-muzero-on-dog_amd/variants
NEW=exploring-muzero-on-dog_amd/libmuz.so
for game in det dog; do
  for rep in 1 2; do
    for lib in $V/libmuz_wseg2048.so $V/libmuz_wseg1024.so $NEW $V/libmuz_wseg256.so; do
      echo "== $game $lib" >> $O/steps.log
      MUZ_LIB=$lib timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game >> $O/steps.log 2>&1 || { tail -20 $O/steps.log; exit 1; }
    done
  done
done
grep -v "^/opt\|amdgpu.ids\|selects" $O/steps.log
for lib in $V/libmuz_convpair0.so $V/libmuz_convpair1.so $NEW; do
  t=$(basename $lib .so)
  MUZ_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/root_$t -o run --output-format csv -- \
    python3 profiles/root_microbench.py 4096 > $O/root_$t.log 2>&1 || { tail -20 $O/root_$t.log; exit 1; }
  find $O/root_$t -name '*kernel_stats.csv' -exec cp {} $O/root_kernel_stats_$t.csv \;
  find $O/root_$t -name '*_kernel_trace.csv' -delete
  echo "== $t"; cut -d, -f1-4 $O/root_kernel_stats_$t.csv | head -4 | cut -c1-40,100-
done
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_nets.py tests/test_gpu_dog_muzero.py \
  tests/test_gpu_selfplay.py tests/test_gpu_stochastic.py tests/test_gpu_headline.py tests/test_gpu_selfplay_classic.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo r6p-done
