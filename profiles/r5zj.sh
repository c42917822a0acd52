#!/bin/bash
# Round 5 end: config (e) train loop lines on HEAD (learner at 69 kernels): det sequential / --overlap, DOG --overlap.
set -o pipefail
O=gpurun_out/r5zj
mkdir -p $O
export TMPDIR=/tmp
for v in "det" "det --overlap" "dog --overlap"; do
  t=$(echo $v | tr -d ' -')
  timeout -k 10 600 python3 bench.py --workload train --game $v --steps 2 --warmup 1 > $O/train_$t.json 2> $O/train_$t.err || { tail -20 $O/train_$t.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/train_$t.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['unit'], d['ms_per_step'])"
done
