#!/bin/bash
# Round 5: k_dog_play per-wave stamps (setup before the check passes, passes, closing-barrier wait) for the lean
# checks and the select-chain checks.
set -o pipefail
O=gpurun_out/r5u
mkdir -p $O
V=$PWD/exploring-muzero-on-dog_amd/variants
for v in dogst dogstnl; do
  MUZ_LIB=$V/libmuz_$v.so timeout -k 10 120 python3 profiles/diag_dog_play_stamps.py > $O/stamps_$v.log 2>&1 || { tail $O/stamps_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/stamps_$v.log
done
