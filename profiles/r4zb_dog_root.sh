#!/bin/bash
# Round 4: k_dog_search compact root (records + the legal slots' noise only) on top of the child records;
# certified interior argmax -- DOG slice parity tests (both tile forms), DOG MuZero bench at the reference's 1500 games
# (one game per wave, then MUZ_DOG_TILE_ROWS=16), stamps in self-play with the exact-path fallback count.
set -o pipefail
O=gpurun_out/r4zb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dog_muzero.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cp gpurun_out/parity.log $O/parity.log 2>/dev/null
timeout -k 10 300 python bench.py --workload dog --policy muzero --steps 3 --warmup 1 > $O/dog_mz.json 2> $O/dog_mz.err || { tail -20 $O/dog_mz.err; exit 1; }
cut -c1-200 $O/dog_mz.json
MUZ_DOG_TILE_ROWS=16 timeout -k 10 300 python bench.py --workload dog --policy muzero --steps 3 --warmup 1 > $O/dog_mz_rows16.json 2> $O/dog_mz_rows16.err || { tail -20 $O/dog_mz_rows16.err; exit 1; }
cut -c1-200 $O/dog_mz_rows16.json
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_st2.so timeout -k 10 300 python profiles/diag_dog_stamps.py selfplay 2>&1 | tee $O/stamps_selfplay.log
