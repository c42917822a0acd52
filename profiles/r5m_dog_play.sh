#!/bin/bash
# Round 5: k_dog_play with closed-form goal cells (dog.hpp dgoal / in_goal_p) against the round-4
# 16-way select chains (-DMUZ_DOG_GOAL_CHAIN=1): DOG GPU tests on the new default, per-wave check-pass stamps of
# both, and the bench (two interleaved repetitions).
set -o pipefail
O=gpurun_out/r5m
mkdir -p $O
V=$PWD/exploring-muzero-on-dog_amd/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_dog.py -x -q --timeout 300 --timeout-method thread > $O/dog_tests.log 2>&1 \
  || { tail -40 $O/dog_tests.log; exit 1; }
tail -2 $O/dog_tests.log
for v in dogst dogst_chain; do
  MUZ_LIB=$V/libmuz_$v.so timeout -k 10 120 python3 profiles/diag_dog_play_stamps.py > $O/stamps_$v.log 2>&1 || { tail $O/stamps_$v.log; exit 1; }
  cat $O/stamps_$v.log
done
for rep in 1 2; do
  for v in chain new; do
    if [ $v = new ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 300 python3 bench.py --workload dog --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$v$rep.json 2> $O/bench_$v$rep.err || { tail $O/bench_$v$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$v$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline'].get('achieved'), d['roofline'].get('frac'))"
  done
done
