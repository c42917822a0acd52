#!/bin/bash
# Round 6: the GPU tests r6m stopped at (the det learner oracle's FLOOR_OK now lists prediction/Dense_5/bias), then
# every root-inference path with the paired conv workgroups; a root kernel trace.
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_learner_oracle.py \
  tests/test_gpu_nets.py tests/test_gpu_dog_muzero.py tests/test_gpu_selfplay.py tests/test_gpu_stochastic.py \
  tests/test_gpu_headline.py tests/test_gpu_selfplay_classic.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
grep "tensors above" $O/tests.log || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/root_trace -o run --output-format csv -- \
  python3 profiles/root_microbench.py 4096 > $O/root_trace.log 2>&1 || { tail -20 $O/root_trace.log; exit 1; }
find $O/root_trace -name '*kernel_stats.csv' -exec cp {} $O/root_kernel_stats.csv \;
find $O/root_trace -name '*_kernel_trace.csv' -delete
head -6 $O/root_kernel_stats.csv | cut -c1-150
echo r6n-done
