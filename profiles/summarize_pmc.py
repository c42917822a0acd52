"""Summarise profiles/pmc_search.sh (three --pmc passes over k_gumbel_search, B = 4096, S = 50) into
profiles/<tag>_pmc.json: per-launch counter means and the derived MFMA / LDS / L2 figures.

    python profiles/summarize_pmc.py <tag>

Derived (MI355X_MICROARCH.md, 'Per-instruction cycle constants' and 'L2'):
  gui_active_cycles = GRBM_GUI_ACTIVE / 8: rocprofv3 sums the GRBM counters over the 8 XCDs (a 3.86-ms
                      launch reads 70.9 M = 8 x 8.86 M cycles at ~2.3 GHz)
  mfma_busy_frac   = SQ_VALU_MFMA_BUSY_CYCLES / (gui_active_cycles x 256 CUs x 4 SIMDs)   (cycles, per SIMD)
  mfma_insts       = SQ_INSTS_VALU_MFMA_F32 (v_mfma_f32_16x16x4_f32, 2048 FLOP each)
  mfma_flop_frac   = mfma_insts x 2048 / (gui_active_cycles x 256 x 256 FLOP/clk/CU)
  l2_hit           = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  lds_conflict     = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE"""
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CUS, SIMDS, XCDS = 256, 4, 8


def passes(src):
    vals = {}
    for f in glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = vals.setdefault(r["Counter_Name"], {})
            d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_pmc")
    mean, n = passes(src)
    gui = mean.get("GRBM_GUI_ACTIVE")
    gui = gui / XCDS if gui else gui
    out = {"kernel": "k_gumbel_search", "workload": "profiles/search_microbench.py 4096 50 (one full-batch search "
           "per launch)", "launches_per_pass": n, "per_launch_mean": mean}
    if gui:
        out["gui_active_cycles"] = gui
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            out["mfma_busy_frac"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * CUS * SIMDS)
        if "SQ_INSTS_VALU_MFMA_F32" in mean:
            out["mfma_flop_frac"] = mean["SQ_INSTS_VALU_MFMA_F32"] * 2048.0 / (gui * CUS * 256.0)
    if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
        out["l2_hit"] = mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"])
    if "SQ_LDS_BANK_CONFLICT" in mean and mean.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_conflict"] = mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_LDS_IDX_ACTIVE"]
    out["source"] = f"profiles/pmc_search.sh {tag} (rocprofv3 --pmc, three separate passes)"
    json.dump(out, open(os.path.join(HERE, f"{tag}_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
