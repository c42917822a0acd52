#!/bin/bash
# Round 4: pinned network rounding (default build) -- parity tests; LayerNorm-on-load / late-heads / split-K logits
# variants -- parity tests and an interleaved A/B (search microbenchmark B=4096 S=50, 3 repetitions).
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
rm -f gpurun_out/parity.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_nets.py tests/test_gpu_headline.py \
  tests/test_gpu_selfplay.py tests/test_gpu_stochastic.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cp gpurun_out/parity.log $O/parity.log
V=$PWD/exploring-muzero-on-dog_amd/variants
for v in lol lhd2k; do
  rm -f gpurun_out/parity.log
  MUZ_LIB=$V/libmuz_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_nets.py \
    tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?
  # 1 = failed assertions (go on to the timing); anything else (time limit, abort, fault) ends the call here
  if [ $rc -ne 0 ]; then tail -40 $O/tests_$v.log; echo "variant $v: pytest rc $rc"; [ $rc -eq 1 ] || exit 1; fi
  tail -2 $O/tests_$v.log
  cp gpurun_out/parity.log $O/parity_$v.log 2>/dev/null
done
for rep in 1 2 3; do
  for v in r3 base pr0 lh d2k lhd2k lol lol2; do
    if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 120 python3 profiles/search_microbench.py 4096 50 2>/dev/null | tee -a $O/ab.log || exit 1
  done
done
unset MUZ_LIB
MUZ_LIB=$V/libmuz_tl.so timeout -k 10 120 python3 profiles/diag_timeline.py 4096 > $O/timeline.log 2>&1 || { tail -20 $O/timeline.log; exit 1; }
cp gpurun_out/timeline.npy $O/timeline.npy
MUZ_LIB=$V/libmuz_tllol.so timeout -k 10 120 python3 profiles/diag_timeline.py 4096 > $O/timeline_lol.log 2>&1 || { tail -20 $O/timeline_lol.log; exit 1; }
cp gpurun_out/timeline.npy $O/timeline_lol.npy
grep -A9 "mean over SIMDs" $O/timeline.log $O/timeline_lol.log
