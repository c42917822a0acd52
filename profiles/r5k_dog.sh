#!/bin/bash
# Round 5: k_dog_play per-wave check-pass stamps; the DOG MuZero line with the C++ slice
# CPU baseline, executed-FLOP frac and PMC traffic.
set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
V=$PWD/exploring-muzero-on-dog_amd/variants
MUZ_LIB=$V/libmuz_dogst.so timeout -k 10 120 python3 profiles/diag_dog_play_stamps.py > $O/dog_play_stamps.log 2>&1 || { tail $O/dog_play_stamps.log; exit 1; }
cat $O/dog_play_stamps.log
timeout -k 10 300 python3 bench.py --workload dog --steps 5 --warmup 1 --no-cpu-baseline > $O/dog_bench.json 2> $O/dog_bench.err || { tail $O/dog_bench.err; exit 1; }
tail -1 $O/dog_bench.json | cut -c1-300
timeout -k 10 400 python3 bench.py --workload dog --policy muzero > $O/dog_mz.json 2> $O/dog_mz.err || { tail $O/dog_mz.err; exit 1; }
tail -1 $O/dog_mz.json | cut -c1-300
