#!/bin/bash
# LDS bank-conflict attribution (verdict r1 item 5): SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE of
#  (1) the isolated MFMA loop (A-fragment ds_read_b128 only; row pad 4 = the search kernel's, 8, 0) and
#  (2) the whole search kernel.  One rocprofv3 --pmc pass per program; summary in gpurun_out/lds_conflicts.log.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lds_pmc
mkdir -p $O
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES"
for v in base pad8 pad0; do
  timeout -k 10 120 rocprofv3 --pmc $C -d $O/lb_$v -o run --output-format csv -- exploring-muzero-on-dog_amd/variants/lb/lb_$v 256 10 > $O/lb_$v.log 2>&1 || { tail -5 $O/lb_$v.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_gumbel_search -d $O/search -o run --output-format csv -- python3 profiles/search_microbench.py 4096 50 > $O/search.log 2>&1 || { tail -5 $O/search.log; exit 1; }
python3 - <<'PY' | tee gpurun_out/lds_conflicts.log
import csv, glob, collections
for name in ["lb_base", "lb_pad8", "lb_pad0", "search"]:
    tot = collections.Counter(); n = set()
    for f in glob.glob(f"gpurun_out/lds_pmc/{name}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r.get("Dispatch_Id"))
    c, a = tot["SQ_LDS_BANK_CONFLICT"], tot["SQ_LDS_IDX_ACTIVE"]
    print(f"{name:8s}: dispatches {len(n)}, LDS instructions {tot['SQ_INSTS_LDS']:.3e}, bank-conflict cycles {c:.3e}, "
          f"LDS active cycles {a:.3e}, conflict share {c / max(a, 1):.3f}, conflict cycles per LDS instruction "
          f"{c / max(tot['SQ_INSTS_LDS'], 1):.2f}")
PY
