"""Summarise profile_workloads.sh runs into profiles/<tag>_<workload>_bench.json and
profiles/<tag>_<workload>_kernel_stats.csv.  Usage: python profiles/summarize_workloads.py <tag>"""
import csv
import glob
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
    for w in (sys.argv[2:] or ("classic", "dog")):
        src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{w}")
        bench = open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1]
        open(os.path.join(HERE, f"{tag}_{w}_bench.json"), "w").write(bench + "\n")
        stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)[0]
        rows = list(csv.DictReader(open(stats)))
        with open(os.path.join(HERE, f"{tag}_{w}_kernel_stats.csv"), "w", newline="") as f:
            out = csv.writer(f)
            out.writerow(["kernel", "calls", "total_ms", "avg_us", "pct", "min_us", "max_us"])
            for r in rows:
                out.writerow([r["Name"].split("(")[0], r["Calls"], f"{float(r['TotalDurationNs']) / 1e6:.3f}",
                              f"{float(r['AverageNs']) / 1e3:.2f}", f"{float(r['Percentage']):.2f}",
                              f"{float(r['MinNs']) / 1e3:.2f}", f"{float(r['MaxNs']) / 1e3:.2f}"])
        print(w, rows[0]["Name"].split("(")[0], rows[0]["AverageNs"])


if __name__ == "__main__":
    main()
