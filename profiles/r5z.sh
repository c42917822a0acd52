#!/bin/bash
# Round 5: learner glue (FiLM reads the batch's action rows in place, im2col reads the transposed observation view in
# place) and the det turn head writing only the read parts of the fp32 root observation: self-play / headline /
# learner GPU tests, learner step time, headline bench.
set -o pipefail
O=gpurun_out/r5z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_headline.py tests/test_gpu_learner.py tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py tests/test_gpu_train_entry.py tests/test_gpu_nets.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 200 python3 profiles/r5_learner_steps.py 30 det > $O/steps_$rep.log 2>&1 || { tail $O/steps_$rep.log; exit 1; }
  grep 'ms per step' $O/steps_$rep.log
done
timeout -k 10 200 python3 profiles/r5_learner_steps.py 30 dog > $O/steps_dog.log 2>&1 || { tail $O/steps_dog.log; exit 1; }
grep 'ms per step' $O/steps_dog.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('headline', d['value'], d['roofline']['end_to_end_frac'])"
bash profiles/r5_learner_trace.sh r5z det > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
head -1 gpurun_out/prof_learner_r5z/step_per_kernel.txt
