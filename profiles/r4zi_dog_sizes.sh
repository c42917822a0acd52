#!/bin/bash
# Round 4: the DOG MuZero line at other batch sizes: 2048 games (one per wave, 256 workgroups: the whole chip) and
# 4096 (two per wave, 256 workgroups).
set -o pipefail
O=gpurun_out/r4zi
mkdir -p $O
for b in 2048 4096; do
  timeout -k 10 400 python bench.py --workload dog --policy muzero --batch $b --steps 2 --warmup 1 --no-cpu-baseline > $O/dog_mz_$b.json 2> $O/dog_mz_$b.err || { tail -20 $O/dog_mz_$b.err; exit 1; }
  cut -c1-200 $O/dog_mz_$b.json
done
