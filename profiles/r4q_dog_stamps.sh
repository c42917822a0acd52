#!/bin/bash
set -o pipefail
O=gpurun_out/r4q
mkdir -p $O
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_st2.so timeout -k 10 300 python profiles/diag_dog_stamps.py selfplay 2>&1 | tee $O/stamps_selfplay.log
