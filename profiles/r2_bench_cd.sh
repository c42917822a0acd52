#!/bin/bash
# Round-2 bench lines for configs (c) and (d), and the DOG actor's per-phase cycle split (diagnostic build).
set -o pipefail
O=gpurun_out/r2_bench
mkdir -p $O
timeout -k 10 500 python bench.py --workload classic --steps 2 --warmup 1 --cpu-seconds 15 > $O/classic.json 2> $O/classic.err || { tail -20 $O/classic.err; exit 1; }
timeout -k 10 300 python bench.py --workload dog --steps 20 --warmup 2 > $O/dog.json 2> $O/dog.err || { tail -20 $O/dog.err; exit 1; }
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_dogst.so timeout -k 10 200 python profiles/diag_dog_stamps.py > $O/dog_stamps.log 2>&1 || { tail -20 $O/dog_stamps.log; exit 1; }
for f in classic dog; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d.get('roofline',{}).get('frac'), d.get('cpu_baseline',{}).get('value'))"; done
cat $O/dog_stamps.log
