#!/bin/bash
# Round 5: k_dog_play phase stamps after the parallel deal.
set -o pipefail
O=gpurun_out/r5zn
mkdir -p $O
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_dogst.so timeout -k 10 120 python3 profiles/diag_dog_play_stamps.py > $O/stamps.log 2>&1 || { tail $O/stamps.log; exit 1; }
grep -v amdgpu.ids $O/stamps.log
