#!/bin/bash
# Round 6 end: the DOG MuZero and classic lines on the final build (their root inference runs k_repr_conv3 too), and the
# det / DOG train iterations (sequential and overlapped).
set -o pipefail
O=gpurun_out/r6aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --workload dog --policy muzero --steps 3 --warmup 1 --no-cpu-baseline > $O/dog_mz.json 2> $O/dog_mz.err || { tail -20 $O/dog_mz.err; exit 1; }
tail -1 $O/dog_mz.json | cut -c1-200
timeout -k 10 400 python3 bench.py --workload classic --no-cpu-baseline > $O/classic.json 2> $O/classic.err || { tail -20 $O/classic.err; exit 1; }
tail -1 $O/classic.json | cut -c1-200
for game in det dog; do
  for ov in "" "--overlap"; do
    tag=${ov:+_overlap}
    timeout -k 10 500 python3 bench.py --workload train --game $game $ov --steps 2 --warmup 1 > $O/train_${game}${tag}.json 2> $O/train_${game}${tag}.err || { tail -20 $O/train_${game}${tag}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/train_${game}${tag}.json').read().strip().splitlines()[-1]); print('$game$tag', d['ms_per_step'], d['roofline']['avg_step_ms'])"
  done
done
echo r6aa-done
