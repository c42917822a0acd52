#!/bin/bash
# Round 5: the DOG train loop with --overlap at 8 vs 6 games per search workgroup (the learner shares the GPU with the
# self-play search: 188 vs 250 CUs held by the search), and the sequential DOG loop at the default.
set -o pipefail
O=gpurun_out/r5zk
mkdir -p $O
export TMPDIR=/tmp
for g in 8 6; do
  MUZ_DOG_GPW=$g timeout -k 10 600 python3 bench.py --workload train --game dog --overlap --steps 2 --warmup 1 > $O/dog_overlap_$g.json 2> $O/dog_overlap_$g.err || { tail -20 $O/dog_overlap_$g.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/dog_overlap_$g.json').read().strip().splitlines()[-1]); print('overlap gpw=$g', d['value'], d['ms_per_step'])"
done
timeout -k 10 600 python3 bench.py --workload train --game dog --steps 2 --warmup 1 > $O/dog_seq.json 2> $O/dog_seq.err || { tail -20 $O/dog_seq.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/dog_seq.json').read().strip().splitlines()[-1]); print('sequential', d['value'], d['ms_per_step'])"
