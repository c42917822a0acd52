#!/bin/bash
# Round-2 (re-entry) profile of HEAD: headline bench + kernel trace + PMC traffic (profile_bench.sh), then a
# kernel trace of the config (e) learner step (graph replay) to rank what remains in it.
set -o pipefail
bash profiles/profile_bench.sh r2c || exit 1
O=gpurun_out/prof_learner_r2c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 profiles/learner_profile.py 20 > $O/learner.log 2>&1 || { tail -20 $O/learner.log; exit 1; }
tail -12 $O/learner.log
# the per-dispatch trace files exceed gpurun's 64 MiB copy-back; the stats summaries are what is kept
find gpurun_out/prof_r2c gpurun_out/prof_learner_r2c -name '*_kernel_trace.csv' -delete
du -sh gpurun_out
