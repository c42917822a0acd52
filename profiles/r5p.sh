#!/bin/bash
# Round 5: (1) FiLM backward without LDS weight staging, scale1 / loss-scale / materialized-zero folds -- learner tests
# + step trace; (2) VERDICT r4 item 5 Option A per-bucket cycles: the search timeline of the dense16 + ln16 build
# (MUZ_LN_EPILOGUE=0) and of dense_ln16 (=1).
set -o pipefail
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_learner_fused.py tests/test_gpu_learner.py tests/test_gpu_learner_oracle.py \
  tests/test_gpu_train_entry.py -x -q --timeout 300 --timeout-method thread > $O/learner_tests.log 2>&1 || { tail -60 $O/learner_tests.log; exit 1; }
tail -1 $O/learner_tests.log
bash profiles/r5_learner_trace.sh r5p det > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
head -14 gpurun_out/prof_learner_r5p/step_per_kernel.txt
V=$PWD/exploring-muzero-on-dog_amd/variants
for v in tl0 tl1; do
  MUZ_LIB=$V/libmuz_$v.so timeout -k 10 120 python3 profiles/diag_timeline.py 4096 > $O/timeline_$v.log 2>&1 || { tail $O/timeline_$v.log; exit 1; }
  grep -A 12 "mean over SIMDs" $O/timeline_$v.log
done
