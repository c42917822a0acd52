#!/bin/bash
# Single-GPU points of the strong-scaling reading (the job's 4096 games split 2048 / 1024 / 512
# per GPU).  Ranks share nothing on the data path, so an N-GPU --split run is N of these side by side.
set -o pipefail
O=gpurun_out/r2c_split
mkdir -p $O
for B in 4096 2048 1024 512; do
  timeout -k 10 300 python bench.py --batch $B --steps 2 --warmup 1 --no-cpu-baseline > $O/b$B.json 2> $O/b$B.err || { tail -20 $O/b$B.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$B.json')); r=d['roofline']; print($B, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])"
done
