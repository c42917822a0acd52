#!/bin/bash
# Round 5: k_dog_search games per workgroup in the one-game-per-wave form (MUZ_DOG_GPW: 8 = 188 workgroups at 1500
# games, 7 = 215, 6 = 250) -- interleaved DOG MuZero bench A/B, then the DOG search / self-play tests at the winner.
set -o pipefail
O=gpurun_out/r5zb
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for gpw in 8 6 7; do
    MUZ_DOG_GPW=$gpw timeout -k 10 300 python3 bench.py --workload dog --policy muzero --steps 2 --warmup 1 --no-cpu-baseline > $O/mz_$gpw$rep.json 2> $O/mz_$gpw$rep.err || { tail $O/mz_$gpw$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/mz_$gpw$rep.json').read().strip().splitlines()[-1]); print('gpw=$gpw', d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
  done
done
MUZ_DOG_GPW=${TEST_GPW:-6} timeout -k 10 600 python -u -m pytest tests/test_gpu_dog_muzero.py tests/test_gpu_dog_records.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
