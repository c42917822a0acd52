#!/bin/bash
# Learner change check: GPU learner tests, then the det step time (graph replay) and the config (e) bench.
set -o pipefail
O=gpurun_out/r2c_learner
mkdir -p $O
export MUZ_PROFILE_DET_ONLY=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python3 profiles/learner_profile.py 100 > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
grep "ms$" $O/profile.log
timeout -k 10 400 python bench.py --workload train --steps 1 --warmup 1 > $O/train.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
cat $O/train.json
