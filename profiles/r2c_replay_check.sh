#!/bin/bash
# Replay ring + learner GPU tests after the sampling-index staging change.
set -o pipefail
O=gpurun_out/r2c_replay
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_learner.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
