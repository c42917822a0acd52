#!/bin/bash
# Round 6: the fused-vs-per-layer learner test with its per-tensor fp32-sensitivity bound, with the split-K Dense_0
# off and on (which tensors need the wider bound, logged); the learner GPU tests; the DOG and det train loops
# overlapped (learner step beside the self-play).
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
export TMPDIR=/tmp
for sk in 0 1; do
  MUZ_SPLITK_DENSE=$sk timeout -k 10 600 python3 -u -m pytest -x -q -s --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_learner_oracle.py -k per_layer > $O/per_layer_sk$sk.log 2>&1 || { tail -40 $O/per_layer_sk$sk.log; exit 1; }
  grep "per-layer path" $O/per_layer_sk$sk.log
done
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner.py \
  tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for game in dog det; do
  timeout -k 10 400 python3 bench.py --workload train --game $game --overlap --steps 2 --warmup 1 \
    > $O/train_${game}_overlap.json 2> $O/train_${game}_overlap.err || { tail -20 $O/train_${game}_overlap.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/train_${game}_overlap.json').read().strip().splitlines()[-1]); print('$game overlap', d['ms_per_step'], d['roofline']['avg_step_ms'])"
done
echo r6s-done
