#!/bin/bash
# Interleaved A/B of k_gumbel_search variants (exploring-muzero-on-dog_amd/variants/libmuz_<v>.so) against the
# in-tree libmuz.so with the search microbenchmark (B=4096, S=50), 3 repetitions:  bash profiles/r3_ab.sh v1 v2 ...
set -o pipefail
O=gpurun_out/ab_r3
mkdir -p $O
for rep in 1 2 3; do
  for v in base "$@"; do
    if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_$v.so; fi
    timeout -k 10 120 python3 profiles/search_microbench.py 4096 50 2>/dev/null | tee -a $O/ab.log || exit 1
  done
done
