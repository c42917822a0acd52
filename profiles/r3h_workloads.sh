#!/bin/bash
# Round 3: HEAD bench lines of the other workloads: classic (config c), DOG (config d, with records + gather),
# config (e) training iteration, env-only micro-benchmark at 4096 and 2^20 games.
set -o pipefail
O=gpurun_out/r3h_workloads
mkdir -p $O
run() { local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python bench.py "$@" > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['unit'], (d.get('roofline') or {}).get('frac'))"; }
run classic 400 --workload classic --steps 2 --warmup 1 --cpu-seconds 15
run dog 300 --workload dog --steps 20 --warmup 2
run dog_records 300 --workload dog --records --steps 20 --warmup 2


run train 400 --workload train --steps 1 --warmup 1
run train_overlap 500 --workload train --overlap --steps 2 --warmup 1
