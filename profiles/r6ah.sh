#!/bin/bash
# Round 6: Dense_0's K split over 4 workgroups per tile (libmuz_d0ks4) against 2 (the build): root kernel traces,
# the root-path GPU tests on the 4-way build, the headline bench for both.
set -o pipefail
O=gpurun_out/r6ah
mkdir -p $O
export TMPDIR=/tmp
V=exploring-muzero-on-dog_amd/variants
NEW=exploring-muzero-on-dog_amd/libmuz.so
for lib in $NEW $V/libmuz_d0ks4.so; do
  t=$(basename $lib .so)
  MUZ_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/root_$t -o run --output-format csv -- \
    python3 profiles/root_microbench.py 4096 > $O/root_$t.log 2>&1 || { tail -20 $O/root_$t.log; exit 1; }
  find $O/root_$t -name '*kernel_stats.csv' -exec cp {} $O/root_kernel_stats_$t.csv \;
  find $O/root_$t -name '*_kernel_trace.csv' -delete
done
python3 - <<'PY'
import csv
for t in ("libmuz", "libmuz_d0ks4"):
    for r in csv.DictReader(open(f"gpurun_out/r6ah/root_kernel_stats_{t}.csv")):
        if "film" not in r["Name"]:
            print(t, r["Name"][:30], round(float(r["AverageNs"]) / 1e3, 1))
PY
MUZ_LIB=$V/libmuz_d0ks4.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_nets.py \
  tests/test_gpu_dog_muzero.py tests/test_gpu_headline.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in $NEW $V/libmuz_d0ks4.so; do
  t=$(basename $lib .so)
  MUZ_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_$t.json 2> $O/bench_$t.err || { tail -20 $O/bench_$t.err; exit 1; }
  tail -1 $O/bench_$t.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$t', d['value'], r['frac'], r['end_to_end_frac'])"
done
echo r6ah-done
