#!/bin/bash
# Round 6: (1) chain / ResBlock-stack row reductions on the DPP / permlane network (MUZ_CHAIN_DPP) against the
# ds_bpermute butterfly -- chain kernels alone, learner steps, learner GPU tests (tolerance-bounded: the summation
# order changed); (2) root inference with two games per conv workgroup (MUZ_CONV_PAIR) -- GPU tests of every root
# path, the root microbenchmark A/B, a kernel trace.
set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
export TMPDIR=/tmp
V=exploring-muzero-on-dog_amd/variants
NEW=exploring-muzero-on-dog_amd/libmuz.so
for rep in 1 2; do
  for lib in $V/libmuz_chaindpp0.so $NEW; do
    echo "== $lib" >> $O/chain_bench.log
    MUZ_LIB=$lib timeout -k 10 180 python3 profiles/chain_bench.py 128 10 20 >> $O/chain_bench.log 2>&1 || { tail -20 $O/chain_bench.log; exit 1; }
  done
done
grep -v "^/opt\|amdgpu.ids\|selects" $O/chain_bench.log
for game in det dog; do
  for lib in $V/libmuz_chaindpp0.so $NEW; do
    echo "== $game $lib" >> $O/steps.log
    MUZ_LIB=$lib timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game >> $O/steps.log 2>&1 || { tail -20 $O/steps.log; exit 1; }
  done
done
grep -v "^/opt\|amdgpu.ids\|selects" $O/steps.log
for rep in 1 2 3; do
  for lib in $V/libmuz_convpair0.so $NEW; do
    MUZ_LIB=$lib timeout -k 10 120 python3 profiles/root_microbench.py 4096 2>&1 | grep root_inference >> $O/root_ab.log || exit 1
  done
done
cat $O/root_ab.log
timeout -k 10 1200 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_nets.py tests/test_gpu_dog_muzero.py \
  tests/test_gpu_selfplay.py tests/test_gpu_stochastic.py tests/test_gpu_headline.py tests/test_gpu_selfplay_classic.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/root_trace -o run --output-format csv -- \
  python3 profiles/root_microbench.py 4096 > $O/root_trace.log 2>&1 || { tail -20 $O/root_trace.log; exit 1; }
find $O/root_trace -name '*kernel_stats.csv' -exec cp {} $O/root_kernel_stats.csv \;
find $O/root_trace -name '*_kernel_trace.csv' -delete
head -6 $O/root_kernel_stats.csv | cut -c1-150
echo r6m-done
