#!/bin/bash
# Round 4: k_gumbel_search with the opaque thread index (MUZ_OPAQUE_TID, 189 VGPRs instead of 215) -- A/B of one
# 4096-game S = 50 search, alternating, 3 reps each.
set -o pipefail
O=gpurun_out/r4zc
mkdir -p $O
for rep in 1 2 3; do
  for v in base tid; do
    if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_$v.so; fi
    echo -n "$v " >> $O/tid_ab.log
    timeout -k 10 120 python3 profiles/search_microbench.py 4096 50 2>/dev/null | tee -a $O/tid_ab.log || exit 1
  done
done
