#!/bin/bash
# Self-play lane kernels as one game per 32 lanes (k_sp_flags_g / k_sp_apply_g): the self-play parity tests, then
# the kernel-trace summary of a one-step headline bench (per-kernel time of a turn).
set -o pipefail
O=gpurun_out/r3_sp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_headline.py tests/test_gpu_reference_api.py \
  tests/test_gpu_env_round.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O -name '*_kernel_trace.csv' -delete
f=$(find $O -name 'run_kernel_stats.csv' | head -1)
head -12 "$f" | cut -d, -f1-5
