#!/bin/bash
# Chain kernels alone (profiles/chain_bench.py): the default build and two timing experiments (row phases
# left out / GEMMs left out), to split a layer's time between its GEMM and its row phase.
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
V=$PWD/exploring-muzero-on-dog_amd/variants
for v in base w16 base w16; do
  if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_ch_$v.so; fi
  echo "== $v"
  timeout -k 10 120 python3 profiles/chain_bench.py 128 10 20 2>/dev/null | tee -a $O/chain_bench.log || exit 1
done
