#!/bin/bash
# Kernel trace of the learner step as the train loop runs it (profiles/r5_learner_steps.py: train_step_from, graph
# replay): the last step's dispatches (after the last k_ring_sample) per kernel and in order.  $1 = tag, $2 = det|dog.
set -o pipefail
O=gpurun_out/prof_learner_${1:-r5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 profiles/r5_learner_steps.py 30 ${2:-det} > $O/learner.log 2>&1 || { tail -20 $O/learner.log; exit 1; }
grep "ms per step" $O/learner.log
python3 - "$O" <<'PY'
import csv, collections, sys, glob
O = sys.argv[1]
f = glob.glob(f"{O}/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
last = max(i for i, r in enumerate(rows) if "k_ring_sample" in r["Kernel_Name"])
step = rows[last:]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
with open(f"{O}/step_sequence.txt", "w") as out:
    out.write(f"# one train_step_from (ring sample + graph replay): {len(step)} kernels, wall {(t1 - t0) / 1e3:.1f} us, "
              f"busy {busy / 1e3:.1f} us\n")
    for r in step:
        out.write(f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.2f} us  {r['Kernel_Name'][:150]}\n")
by, t = collections.Counter(), collections.Counter()
for r in step:
    n = r["Kernel_Name"].split("(")[0][:120]
    by[n] += 1
    t[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
with open(f"{O}/step_per_kernel.txt", "w") as out:
    out.write(f"# one train_step_from: {len(step)} kernels, wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us\n")
    for n, c in sorted(t.items(), key=lambda x: -x[1]):
        out.write(f"{by[n]:5d} {c / 1e3:9.1f} us {c / by[n] / 1e3:7.2f} us/call  {n}\n")
PY
find $O -name '*_kernel_trace.csv' -delete
head -1 $O/step_per_kernel.txt
