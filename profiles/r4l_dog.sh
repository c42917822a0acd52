#!/bin/bash
# Round 4: k_dog_search with {prior, value, reward, discount} child records and batched loads -- DOG slice tests +
# bench + timing variants.
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dog_muzero.py -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$PWD/exploring-muzero-on-dog_amd/variants
for v in base FASTEXP; do
  if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_dog_$v.so; fi
  timeout -k 10 200 python bench.py --workload dog --policy muzero --steps 1 --warmup 0 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$v.json')); print('$v', d['value'], d['roofline']['avg_launch_ms'])" | tee -a $O/ab.log
done
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_st2.so timeout -k 10 200 python profiles/diag_dog_stamps.py 1024 100 50 2>&1 | tee $O/stamps.log
