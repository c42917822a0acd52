#!/bin/bash
# Env round kernels, round 3 (second pass): oracle parity of every variant, then --workload env at 4096 / 65536 /
# 2^20 games with each kernel (1 = one game per lane, 2 / 3 / 4 / 5 = one game per 32 / 8 / 4 / 16 lanes).
set -o pipefail
O=gpurun_out/${ENV_OUT:-r3_env2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_env_round.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for B in ${ENV_BATCHES:-4096 65536 1048576}; do
  for v in ${ENV_VARIANTS:-1 2 3 4 5}; do
    timeout -k 10 300 python bench.py --workload env --batch $B --env-variant $v --steps 3 --warmup 1 --no-cpu-baseline \
      > $O/env_${B}_v$v.json 2> $O/env_${B}_v$v.err || { tail -20 $O/env_${B}_v$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/env_${B}_v$v.json')); r=d['roofline']; print($B, $v, d['value'], r['kernel'], r['avg_launch_ms'], r['frac'])" | tee -a $O/summary.txt
  done
done
