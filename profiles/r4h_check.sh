#!/bin/bash
# Round 4: (1) the generalised chain kernels (8 waves default; 16-wave build) -- chain tests + micro-bench A/B;
# (2) the search ring's two accumulation chains per tile (-DMUZ_ACC_CHAINS=2) -- parity tests + interleaved A/B.
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
V=$PWD/exploring-muzero-on-dog_amd/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -q -k "chain" --timeout 200 --timeout-method thread > $O/chain_tests.log 2>&1 \
  || { tail -30 $O/chain_tests.log; exit 1; }
tail -1 $O/chain_tests.log
MUZ_LIB=$V/libmuz_ch_w16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -q -k "chain_kernel" --timeout 200 \
  --timeout-method thread > $O/chain_tests_w16.log 2>&1; rc=$?
tail -1 $O/chain_tests_w16.log; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in base w16; do
    if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_ch_$v.so; fi
    echo "== $v" | tee -a $O/chain_bench.log
    timeout -k 10 120 python3 profiles/chain_bench.py 128 10 20 2>/dev/null | tee -a $O/chain_bench.log || exit 1
  done
done
unset MUZ_LIB
MUZ_LIB=$V/libmuz_acc2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_nets.py tests/test_gpu_headline.py \
  -x -q --timeout 300 --timeout-method thread > $O/tests_acc2.log 2>&1; rc=$?
tail -1 $O/tests_acc2.log; [ $rc -le 1 ] || exit 1
for rep in 1 2 3; do
  for v in base acc2; do
    if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 120 python3 profiles/search_microbench.py 4096 50 2>/dev/null | tee -a $O/ab.log || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner_fused.py tests/test_gpu_learner.py tests/test_gpu_learner_oracle.py -x -q \
  --timeout 300 --timeout-method thread > $O/learner_tests.log 2>&1 || { tail -30 $O/learner_tests.log; exit 1; }
tail -1 $O/learner_tests.log
timeout -k 10 600 python3 profiles/learner_profile.py 50 > $O/learner_profile.log 2>&1 || { tail -20 $O/learner_profile.log; exit 1; }
grep "ms$" $O/learner_profile.log
