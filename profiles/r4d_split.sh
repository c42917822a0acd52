#!/bin/bash
# Round 4 verdict item 3: a 16-game tile on one CU vs split over two CUs of one XCD with a per-layer L2 exchange
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
for t in 32 64 128; do
  for m in 0 2 1; do
    timeout -k 5 60 ./profiles/split_tile_bench $t $m 20 | tee -a $O/split_tile.log || exit 1
  done
done
