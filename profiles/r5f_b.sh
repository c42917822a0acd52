#!/bin/bash
# Round 5 final, part B: the other workload lines (default flags): DOG MuZero self-play at 1500 games, DOG random
# policy, classic MADN, and the DOG train loop (--overlap).
set -o pipefail
O=gpurun_out/${R5F_OUT:-r5f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --workload dog --policy muzero > $O/dog_mz.json 2> $O/dog_mz.err || { tail -20 $O/dog_mz.err; exit 1; }
cut -c1-300 $O/dog_mz.json
timeout -k 10 300 python3 bench.py --workload dog > $O/dog.json 2> $O/dog.err || { tail -20 $O/dog.err; exit 1; }
cut -c1-300 $O/dog.json
timeout -k 10 400 python3 bench.py --workload classic > $O/classic.json 2> $O/classic.err || { tail -20 $O/classic.err; exit 1; }
cut -c1-300 $O/classic.json
