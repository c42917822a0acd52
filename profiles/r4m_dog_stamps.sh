#!/bin/bash
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_st2.so timeout -k 10 200 python profiles/diag_dog_stamps.py 1024 100 50 2>&1 | tee $O/stamps.log
