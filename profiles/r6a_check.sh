#!/bin/bash
# round 6, first GPU call: the tests this round changed + the config (e) parts measurement
set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_learner.py tests/test_gpu_learner_fused.py tests/test_gpu_reference_api.py \
  tests/test_gpu_dog_records.py tests/test_gpu_replay.py > gpurun_out/r6a/tests.log 2>&1 || { tail -30 gpurun_out/r6a/tests.log; exit 1; }
tail -3 gpurun_out/r6a/tests.log
timeout -k 10 600 python -u profiles/config_e_parts.py det dog > gpurun_out/r6a/parts.log 2>&1 || { tail -30 gpurun_out/r6a/parts.log; exit 1; }
tail -3 gpurun_out/r6a/parts.log
