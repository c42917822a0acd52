"""Summarise a profile_bench.sh run (gpurun_out/prof_<tag>) into committed files under profiles/:
  <tag>_bench.json          the bench line of that run
  <tag>_kernel_stats.csv    rocprofv3 --kernel-trace --stats summary (names shortened)
  <tag>_traffic.json        PMC HBM bytes per k_gumbel_search launch (FETCH_SIZE doubled per the gfx950
                            note, + WRITE_SIZE, both KB -> bytes), read by bench.py as roofline.traffic
Usage: python profiles/summarize_profile.py <tag>"""
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def counter_total(pattern, name):
    vals = {}
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return vals


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    bench = open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1]
    open(os.path.join(HERE, f"{tag}_bench.json"), "w").write(bench + "\n")
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(stats)))
    with open(os.path.join(HERE, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_us", "pct", "min_us", "max_us"])
        for r in rows:
            w.writerow([r["Name"].split("(")[0], r["Calls"], f"{float(r['TotalDurationNs']) / 1e6:.3f}",
                        f"{float(r['AverageNs']) / 1e3:.2f}", f"{float(r['Percentage']):.2f}",
                        f"{float(r['MinNs']) / 1e3:.2f}", f"{float(r['MaxNs']) / 1e3:.2f}"])
    fetch = counter_total(os.path.join(src, "pmc_fetch", "**", "*counter_collection.csv"), "FETCH_SIZE")
    write = counter_total(os.path.join(src, "pmc_write", "**", "*counter_collection.csv"), "WRITE_SIZE")
    n_f, n_w = max(1, len(fetch)), max(1, len(write))
    fetch_b = 2.0 * 1024.0 * sum(fetch.values()) / n_f    # gfx950: FETCH_SIZE counts half of a wide stream
    write_b = 1024.0 * sum(write.values()) / n_w
    search = [r for r in rows if r["Name"].startswith("muz::k_gumbel_search")][0]
    out = {"kernel": "k_gumbel_search", "launches_fetch_pass": len(fetch), "launches_write_pass": len(write),
           "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
           "bytes_per_launch": fetch_b + write_b,
           "avg_launch_us_trace": float(search["AverageNs"]) / 1e3,
           "source": f"profiles/profile_bench.sh {tag} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)"}
    json.dump(out, open(os.path.join(HERE, f"{tag}_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
