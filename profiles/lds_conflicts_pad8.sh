set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lds_pmc8
mkdir -p $O
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_pad8.so timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-include-regex k_gumbel_search -d $O/search -o run --output-format csv -- python3 profiles/search_microbench.py 4096 50 > $O/search.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
tot = collections.Counter(); n=set()
for f in glob.glob("gpurun_out/lds_pmc8/search/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r.get("Dispatch_Id"))
c, a = tot["SQ_LDS_BANK_CONFLICT"], tot["SQ_LDS_IDX_ACTIVE"]
print(f"search pad8: dispatches {len(n)}, LDS instructions {tot['SQ_INSTS_LDS']:.3e}, bank-conflict cycles {c:.3e}, LDS active {a:.3e}, share {c/max(a,1):.3f}")
PY
