#!/bin/bash
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_random_start.py tests/test_gpu_env.py tests/test_gpu_env_round.py tests/test_gpu_dog.py \
  tests/test_gpu_classic.py tests/test_gpu_dog_muzero.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
