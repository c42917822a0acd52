#!/bin/bash
# Round 6: the learner GPU tests with the split-K Dense_0 off (default), the det / DOG learner steps, and the DOG / det
# train loops with --overlap (the learner step beside the self-play: VERDICT r5 item 7's DOG <= 2.1 ms).
set -o pipefail
O=gpurun_out/r6u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for game in det dog; do
    timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game 2>&1 | grep "ms per step" >> $O/steps.log || exit 1
  done
done
cat $O/steps.log
for game in dog det; do
  timeout -k 10 400 python3 bench.py --workload train --game $game --overlap --steps 2 --warmup 1 \
    > $O/train_${game}_overlap.json 2> $O/train_${game}_overlap.err || { tail -20 $O/train_${game}_overlap.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/train_${game}_overlap.json').read().strip().splitlines()[-1]); print('$game overlap', d['ms_per_step'], d['roofline']['avg_step_ms'])"
done
echo r6u-done
