#!/bin/bash
# Round 4: DOG MuZero slice (encode, nets at A = 806, search) + the det nets / search after the repr16 refactor.
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dog_muzero.py tests/test_gpu_nets.py tests/test_gpu_search.py -v \
  --timeout 200 --timeout-method thread -s > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|dog root|dog recurrent|Error" $O/tests.log | head -40; tail -3 $O/tests.log
cp gpurun_out/parity.log $O/ 2>/dev/null

[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload dog --policy muzero --steps 2 --warmup 1 > $O/dog_mz_bench.json 2> $O/dog_mz_bench.err \
  || { tail -20 $O/dog_mz_bench.err; exit 1; }
cut -c1-900 $O/dog_mz_bench.json
