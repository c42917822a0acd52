#!/bin/bash
# Kernel trace of the det learner step alone (graph replay, batch 128 / unroll 10): per-kernel totals and the
# ordered kernel sequence of ONE replayed step (what a fused learner has to replace).
set -o pipefail
O=gpurun_out/prof_learner_r3${1:+_$1}
mkdir -p $O
export TMPDIR=/tmp MUZ_PROFILE_DET_ONLY=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 profiles/learner_profile.py 50 > $O/learner.log 2>&1 || { tail -20 $O/learner.log; exit 1; }
grep "ms$" $O/learner.log
python3 - "$O" <<'PY'
import csv, collections, sys, glob
O = sys.argv[1]
f = glob.glob(f"{O}/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the last 50 dispatch groups are graph replays of "sample_batch + train_step"; take the final step: the
# dispatches after the last k_ring_sample
last = max(i for i, r in enumerate(rows) if "k_ring_sample" in r["Kernel_Name"])
step = rows[last:]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
with open(f"{O}/step_sequence.txt", "w") as out:
    out.write(f"# one sample + train step: {len(step)} kernels, wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us\n")
    for r in step:
        out.write(f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.2f} us  {r['Kernel_Name'][:110]}\n")
by, t = collections.Counter(), collections.Counter()
for r in step:
    n = r["Kernel_Name"].split("(")[0][:90]
    by[n] += 1
    t[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
with open(f"{O}/step_per_kernel.txt", "w") as out:
    for n, c in sorted(t.items(), key=lambda x: -x[1]):
        out.write(f"{by[n]:5d} {c / 1e3:9.1f} us {c / by[n] / 1e3:7.2f} us/call  {n}\n")
PY
find $O -name '*_kernel_trace.csv' -delete
head -3 $O/step_sequence.txt
head -40 $O/step_per_kernel.txt
