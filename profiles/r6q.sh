#!/bin/bash
# Round 6: learner step traces (det, DOG) with the DPP row sums, the narrow fused forward and 256-row weight-gradient
# segments; then the whole GPU suite on this build.
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
bash profiles/r5_learner_trace.sh r6q_det det || exit 1
bash profiles/r5_learner_trace.sh r6q_dog dog || exit 1
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo r6q-done
