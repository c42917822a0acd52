#!/bin/bash
# Round 5: k_dog_play's per-turn random draw computed by wave 3 during the checks (off wave 0's serial pick) -- DOG
# GPU tests (bit-exact vs the oracle), then an interleaved bench A/B against HEAD (variants/libmuz_u0.so).
set -o pipefail
O=gpurun_out/r5zo
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "dog" --timeout 300 --timeout-method thread > $O/dog_tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/dog_tests.log | head -20; tail -3 $O/dog_tests.log; exit 1; }
tail -1 $O/dog_tests.log
V=$PWD/exploring-muzero-on-dog_amd/variants
for rep in 1 2; do
  for v in u0 new; do
    if [ $v = new ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 300 python3 bench.py --workload dog --steps 5 --warmup 1 --no-cpu-baseline > $O/dog_$v$rep.json 2> $O/dog_$v$rep.err || { tail $O/dog_$v$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/dog_$v$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline'].get('achieved'))"
  done
done
