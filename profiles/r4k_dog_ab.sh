#!/bin/bash
# Round 4: where k_dog_search's time goes -- timing variants (wrong results, experiments only): float exp instead of
# the correctly rounded double exp; no walk at all (fixed child, no node loads).
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
V=$PWD/exploring-muzero-on-dog_amd/variants
for v in base NOBAR FASTEXP_NOBAR LOADONLY; do
  if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_dog_$v.so; fi
  timeout -k 10 200 python bench.py --workload dog --policy muzero --steps 1 --warmup 0 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$v.json')); print('$v', d['value'], d['roofline']['avg_launch_ms'])" | tee -a $O/ab.log
done
