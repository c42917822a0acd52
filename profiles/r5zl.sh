#!/bin/bash
# Round 5: the DOG train loop with --overlap at the code's own setting (no MUZ_DOG_GPW in the environment).
set -o pipefail
O=gpurun_out/r5zl
mkdir -p $O
export TMPDIR=/tmp
unset MUZ_DOG_GPW
timeout -k 10 600 python3 bench.py --workload train --game dog --overlap --steps 2 --warmup 1 > $O/dog_overlap.json 2> $O/dog_overlap.err || { tail -20 $O/dog_overlap.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/dog_overlap.json').read().strip().splitlines()[-1]); print('overlap', d['value'], d['ms_per_step'])"
