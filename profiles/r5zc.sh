#!/bin/bash
# Round 5: k_dog_search compact-walk changes (visited-slot words by LDS or, exp(prior - pm) computed once per visited
# child) -- DOG search / self-play GPU tests (bit-identical), then an interleaved DOG MuZero A/B against HEAD's build
# (variants/libmuz_walk0.so).
set -o pipefail
O=gpurun_out/r5zc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "dog" --timeout 300 --timeout-method thread > $O/dog_tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/dog_tests.log | head -20; tail -3 $O/dog_tests.log; exit 1; }
tail -1 $O/dog_tests.log
V=$PWD/exploring-muzero-on-dog_amd/variants
for rep in 1 2; do
  for v in walk0 new; do
    if [ $v = new ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 300 python3 bench.py --workload dog --policy muzero --steps 2 --warmup 1 --no-cpu-baseline > $O/mz_$v$rep.json 2> $O/mz_$v$rep.err || { tail $O/mz_$v$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/mz_$v$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
  done
done
