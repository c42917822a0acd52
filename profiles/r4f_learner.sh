#!/bin/bash
# Round 4 verdict item 4: the learner's dynamics chain as one launch each way (csrc/learner_chain.hip) --
# learner GPU tests (chain kernel against the per-layer path and per-step autograd, oracle steps), step times
# with the chain kernel on / off, and a kernel trace of one det step (kernel count against round 3's 408).
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_learner_fused.py tests/test_gpu_learner_oracle.py \
  -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 profiles/learner_profile.py 50 > $O/learner_profile.log 2>&1 || { tail -20 $O/learner_profile.log; exit 1; }
cat $O/learner_profile.log | grep "ms$"
timeout -k 10 400 bash profiles/r3_learner_trace.sh r4 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cat $O/trace.log
cp gpurun_out/prof_learner_r3_r4/step_sequence.txt $O/ 2>/dev/null
cp gpurun_out/prof_learner_r3_r4/step_per_kernel.txt $O/ 2>/dev/null
