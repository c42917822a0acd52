#!/bin/bash
# Round 6: root inference with the padded conv rows (k_repr_conv) and Dense_0 as one L2-tiled GEMM (k_dense0):
# GPU tests of everything that runs root inference, the root microbenchmark A/B against the round-6 base build
# (3 interleaved repetitions), a kernel trace of the new root, and the MFMA rounding probe.
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_nets.py \
  tests/test_gpu_dog_muzero.py tests/test_gpu_selfplay.py tests/test_gpu_stochastic.py tests/test_gpu_headline.py \
  tests/test_gpu_selfplay_classic.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
V=$PWD/exploring-muzero-on-dog_amd/variants
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = new ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_r6base.so; fi
    timeout -k 10 120 python3 profiles/root_microbench.py 4096 2>&1 | grep root_inference >> $O/root_ab.log || exit 1
  done
done
unset MUZ_LIB
cat $O/root_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/root_trace -o run --output-format csv -- \
  python3 profiles/root_microbench.py 4096 > $O/root_trace.log 2>&1 || { tail -20 $O/root_trace.log; exit 1; }
find $O/root_trace -name '*kernel_stats.csv' -exec cp {} $O/root_kernel_stats.csv \;
find $O/root_trace -name '*_kernel_trace.csv' -delete
head -6 $O/root_kernel_stats.csv | cut -c1-150
timeout -k 10 300 python3 profiles/mfma_rounding.py 300 > $O/mfma_rounding.log 2>&1 || { tail -20 $O/mfma_rounding.log; exit 1; }
cat $O/mfma_rounding.log
echo r6c-done
