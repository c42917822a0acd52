#!/bin/bash
# Round 5: where the DOG MuZero bench's GPU idles between turns (~2.8 ms of a 22.9 ms turn): kernel trace + HIP
# runtime trace of one bench step; per-turn gaps and the slowest host API calls summarised.
set -o pipefail
O=gpurun_out/r5ze
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $O/tr -o run --output-format csv -- \
  python3 bench.py --workload dog --policy muzero --steps 1 --warmup 1 --no-cpu-baseline > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
k = sorted(csv.DictReader(open(glob.glob(f"{O}/tr/**/*kernel_trace.csv", recursive=True)[0])), key=lambda r: int(r["Start_Timestamp"]))
print("kernels", len(k))
gaps = sorted(((int(b["Start_Timestamp"]) - int(a["End_Timestamp"]), a["Kernel_Name"][:40], b["Kernel_Name"][:40])
               for a, b in zip(k, k[1:])), reverse=True)
for g, x, y in gaps[:8]:
    print(f"gap {g / 1e3:9.1f} us after {x} before {y}")
print("total gap us", sum(g[0] for g in gaps) / 1e3, "span us", (int(k[-1]["End_Timestamp"]) - int(k[0]["Start_Timestamp"])) / 1e3)
h = sorted(csv.DictReader(open(glob.glob(f"{O}/tr/**/*hip_api_trace.csv", recursive=True)[0])), key=lambda r: int(r["Start_Timestamp"]))
launches = [r for r in h if r["Function"] == "hipLaunchKernel"]
print("launch calls", len(launches), "kernel dispatches", len(k))
# launches and dispatches in submission order: the slowest launch calls with the kernel they submitted
for r, kk in sorted(zip(launches, k), key=lambda p: -(int(p[0]["End_Timestamp"]) - int(p[0]["Start_Timestamp"])))[:10]:
    print(f"launch {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:9.1f} us  {kk['Kernel_Name'][:60]}")
PY
find $O/tr -name '*_trace.csv' -delete
