#!/bin/bash
# round 6, first GPU call: the tests this round changed, the DOG search with the visited-mask tree (tests + bench A/B
# against the round-5 library), and the config (e) parts measurement.
# (first pass, same tree: test_gpu_dog_muzero / learner / learner_fused / reference_api / dog_records / replay -- 103
# passed, the learner oracle's new per-tensor bound then named the classic discount head: FLOOR_OK)
set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_learner_oracle.py > gpurun_out/r6a/tests2.log 2>&1 || { tail -30 gpurun_out/r6a/tests2.log; exit 1; }
tail -3 gpurun_out/r6a/tests2.log
for lib in exploring-muzero-on-dog_amd/variants/libmuz_r5.so exploring-muzero-on-dog_amd/libmuz.so; do
  MUZ_LIB=$lib timeout -k 10 300 python -u bench.py --workload dog --policy muzero --steps 4 --warmup 1 --no-cpu-baseline >> gpurun_out/r6a/dog_mz.log 2>&1 || { tail -30 gpurun_out/r6a/dog_mz.log; exit 1; }
done
tail -2 gpurun_out/r6a/dog_mz.log
timeout -k 10 600 python -u profiles/config_e_parts.py det dog > gpurun_out/r6a/parts.log 2>&1 || { tail -30 gpurun_out/r6a/parts.log; exit 1; }
tail -3 gpurun_out/r6a/parts.log
