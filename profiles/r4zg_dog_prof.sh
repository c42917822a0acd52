#!/bin/bash
# Round 4: rocprofv3 kernel stats of the DOG MuZero bench line (k_dog_search's launches against the line's
# avg_launch_ms, which times the launches of the timed steps only; the warmup turns' launches are shorter).
set -o pipefail
O=gpurun_out/r4zg
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload dog --policy muzero --steps 2 --warmup 1 --no-cpu-baseline > $O/dog_mz_prof.json 2> $O/dog_mz_prof.err || { tail -20 $O/dog_mz_prof.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
python3 - "$O" <<'PY'
import csv, glob, json, sys
O = sys.argv[1]
rows = [r for f in glob.glob(f"{O}/prof/**/*_kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
ds = sorted((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
            for r in rows if "k_dog_search" in r["Kernel_Name"])
d = [x for _, x in ds]
line = json.load(open(f"{O}/dog_mz_prof.json"))
out = {"launches": len(d), "all_avg_ms": sum(d) / len(d), "last16_avg_ms": sum(d[-16:]) / 16,
       "first9_avg_ms": sum(d[:9]) / 9, "bench_avg_launch_ms": line["roofline"]["avg_launch_ms"], "per_launch_ms": d}
json.dump(out, open(f"{O}/dog_search_launches.json", "w"), indent=1)
print({k: v for k, v in out.items() if k != "per_launch_ms"})
PY
find $O/prof -name '*_kernel_trace.csv' -delete
