"""HBM bytes per launch of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs), with
the MI355X_MICROARCH.md corrections summarize_profile.py applies: both counters are KB, FETCH_SIZE doubled on gfx950.

usage: python profiles/summarize_pmc_kernel.py <fetch_dir> <write_dir> <kernel substring> <source text> > out.json
"""
import csv
import glob
import json
import os
import sys


def per_launch(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    fdir, wdir, kernel, source = sys.argv[1:5]
    f, w = per_launch(fdir, "FETCH_SIZE", kernel), per_launch(wdir, "WRITE_SIZE", kernel)
    if not f or not w:
        raise SystemExit(f"no {kernel} launches in {fdir} / {wdir}")
    fb = 2.0 * 1024.0 * sum(f) / len(f)
    wb = 1024.0 * sum(w) / len(w)
    print(json.dumps({"kernel": kernel, "launches_fetch_pass": len(f), "launches_write_pass": len(w),
                      "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb, "bytes_per_launch": fb + wb,
                      "source": source}, indent=1))


if __name__ == "__main__":
    main()
