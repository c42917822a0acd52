#!/bin/bash
# Round 5: (1) learner FiLM kernels rewritten (float4 LDS reads, split columns) -- FiLM tests + step trace;
# (2) VERDICT r4 item 5 Option A (nn.hpp dense_ln16: LayerNorm statistics in the dense epilogue, variant
# libmuz_lne.so) -- parity tests on the variant, then the search microbenchmark A/B (B=4096 S=50, 3 interleaved reps).
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner_fused.py -x -q -k "film" --timeout 200 --timeout-method thread > $O/film_tests.log 2>&1 || { tail -40 $O/film_tests.log; exit 1; }
tail -1 $O/film_tests.log
bash profiles/r5_learner_trace.sh r5o det > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
head -12 gpurun_out/prof_learner_r5o/step_per_kernel.txt
V=$PWD/exploring-muzero-on-dog_amd/variants
rm -f gpurun_out/parity.log
MUZ_LIB=$V/libmuz_lne.so timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_nets.py tests/test_gpu_headline.py \
  tests/test_gpu_selfplay.py tests/test_gpu_stochastic.py tests/test_gpu_dog_muzero.py -x -q --timeout 300 --timeout-method thread > $O/tests_lne.log 2>&1
rc=$?
tail -3 $O/tests_lne.log
cp gpurun_out/parity.log $O/parity_lne.log 2>/dev/null
if [ $rc -ne 0 ]; then tail -40 $O/tests_lne.log; [ $rc -eq 1 ] || exit 1; fi
for rep in 1 2 3; do
  for v in base lne; do
    if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 120 python3 profiles/search_microbench.py 4096 50 2>/dev/null | sed "s/^/$v /" | tee -a $O/ab.log || exit 1
  done
done
unset MUZ_LIB
