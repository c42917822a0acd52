#!/bin/bash
# Kernel trace of the det learner step alone (graph replay, batch 128 / unroll 10): which kernels the 3.4 ms go to.
set -o pipefail
O=gpurun_out/prof_learner_det_r2c
mkdir -p $O
export TMPDIR=/tmp MUZ_PROFILE_DET_ONLY=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 profiles/learner_profile.py 200 > $O/learner.log 2>&1 || { tail -20 $O/learner.log; exit 1; }
grep "ms$" $O/learner.log
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/prof_learner_det_r2c/trace/run_kernel_trace.csv")))
# the graph replays of the last 200 + 200 steps: keep dispatches after the first sample_batch timing window
by = collections.Counter(); t = collections.Counter()
for r in rows:
    n = r["Kernel_Name"]
    by[n] += 1
    t[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
with open("gpurun_out/prof_learner_det_r2c/per_kernel.txt", "w") as f:
    for n, c in sorted(t.items(), key=lambda x: -x[1])[:60]:
        f.write(f"{by[n]:7d} {c/1e6:9.2f} ms {c/by[n]/1e3:8.2f} us  {n[:120]}\n")
PY
find $O -name '*_kernel_trace.csv' -delete
head -40 $O/per_kernel.txt
