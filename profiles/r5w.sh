#!/bin/bash
# Round 5: k_dog_search cycle shares over DogSelfPlay turns (B=1500, S=100, D=50) on HEAD, with the first-walk
# normaliser / top-prior work as its own category and the full-load / first-walk counts.
set -o pipefail
O=gpurun_out/r5w
mkdir -p $O
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_st2.so timeout -k 10 300 python3 profiles/diag_dog_stamps.py selfplay > $O/stamps_selfplay.log 2>&1 || { tail $O/stamps_selfplay.log; exit 1; }
grep -v amdgpu.ids $O/stamps_selfplay.log
