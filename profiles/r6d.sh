#!/bin/bash
# Round 6: k_dense0 tiling variants (MUZ_D0_NG column groups per workgroup x MUZ_D0_KC k-blocks per chunk) and the
# conv0 register-weights change: root kernel traces per variant (per-kernel averages), the root microbenchmark, and
# the root / nets tests on the default build; then the r6b measurements (classic eval tests, PMC traffic, traces).
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_nets.py \
  tests/test_gpu_dog_muzero.py -k "root or nets or network or recurrent" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$PWD/exploring-muzero-on-dog_amd/variants
for v in default d0_2_8 d0_1_4 d0_1_8; do
  if [ $v = default ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$v -o run --output-format csv -- \
    python3 profiles/root_microbench.py 4096 > $O/trace_$v.log 2>&1 || { tail -20 $O/trace_$v.log; exit 1; }
  grep root_inference $O/trace_$v.log
  f=$(find $O/trace_$v -name '*kernel_stats.csv' | head -1)
  grep -E "k_dense0|k_repr_conv|k_root_dense" $f | awk -F, -v v=$v '{printf "%s %s avg %.1f us\n", v, $1, $4/1000}'
  find $O/trace_$v -name '*_kernel_trace.csv' -delete
done
unset MUZ_LIB
echo r6d-done
