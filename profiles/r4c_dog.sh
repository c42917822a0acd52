#!/bin/bash
# Round 4: DOG play-phase env_step on wave 0's 64 lanes -- DOG GPU tests, stamp shares (new vs lane-0 step), bench.
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dog.py -x -q --timeout 300 --timeout-method thread > $O/dog_tests.log 2>&1 \
  || { tail -40 $O/dog_tests.log; exit 1; }
tail -2 $O/dog_tests.log
V=$PWD/exploring-muzero-on-dog_amd/variants
MUZ_LIB=$V/libmuz_dogst.so timeout -k 10 120 python3 profiles/diag_dog_stamps.py > $O/dog_stamps_wave.log 2>&1 || { tail $O/dog_stamps_wave.log; exit 1; }
MUZ_LIB=$V/libmuz_dogst0.so timeout -k 10 120 python3 profiles/diag_dog_stamps.py > $O/dog_stamps_lane0.log 2>&1 || { tail $O/dog_stamps_lane0.log; exit 1; }
tail -8 $O/dog_stamps_wave.log $O/dog_stamps_lane0.log
for rep in 1 2; do
  for v in r3 new; do
    if [ $v = new ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 300 python3 bench.py --workload dog --steps 5 --warmup 1 --no-cpu-baseline > $O/dog_bench_$v$rep.json 2> $O/dog_bench_$v$rep.err || { tail $O/dog_bench_$v$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/dog_bench_$v$rep.json')); print('$v', d['value'], d['roofline'].get('achieved'), d['roofline'].get('frac'))"
  done
done
