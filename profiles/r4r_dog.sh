#!/bin/bash
# Round 4: k_dog_search with per-node cached prior normalisers -- DOG slice tests, bench, stamps in self-play.
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dog_muzero.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --workload dog --policy muzero --steps 3 --warmup 1 > $O/dog_mz.json 2> $O/dog_mz.err || { tail -20 $O/dog_mz.err; exit 1; }
cut -c1-200 $O/dog_mz.json
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_st2.so timeout -k 10 300 python profiles/diag_dog_stamps.py selfplay 2>&1 | tee $O/stamps_selfplay.log
