#!/bin/bash
# Learner after the LayerNorm_0 + FiLM fusion: its GPU tests (kernels vs float64 autograd, chain node vs per-step
# autograd, device learner vs the oracle at config (e) shape), the per-step kernel trace, the config (e) benches.
set -o pipefail
O=gpurun_out/r3_learner
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py \
  tests/test_gpu_train_entry.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash profiles/r3_learner_trace.sh r3e || exit 1
timeout -k 10 400 python bench.py --workload train --steps 1 --warmup 1 > $O/train.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
timeout -k 10 500 python bench.py --workload train --overlap --steps 2 --warmup 1 > $O/train_overlap.json 2> $O/train_overlap.err || { tail -20 $O/train_overlap.err; exit 1; }
python3 -c "
import json
for n in ('train', 'train_overlap'):
    d = json.load(open('$O/' + n + '.json')); print(n, d['value'], d['ms_per_step'], d['roofline']['avg_step_ms'])"
