#!/bin/bash
# Round-2 bench lines: headline det (config b), classic (config c) with roofline + CPU baseline, DOG (config d).
set -o pipefail
O=gpurun_out/r2_bench
mkdir -p $O
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > $O/det.json 2> $O/det.err || { tail -20 $O/det.err; exit 1; }
timeout -k 10 400 python bench.py --workload classic --steps 2 --warmup 1 --cpu-seconds 15 > $O/classic.json 2> $O/classic.err || { tail -20 $O/classic.err; exit 1; }
timeout -k 10 300 python bench.py --workload dog --steps 20 --warmup 2 > $O/dog.json 2> $O/dog.err || { tail -20 $O/dog.err; exit 1; }
for f in det classic dog; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d.get('roofline',{}).get('frac'), d.get('cpu_baseline',{}).get('value'))"; done
