#!/bin/bash
# Round 6: the paired conv kernel with register-resident LayerNorms (k_repr_conv3, 4 pairs per CU) against the
# 4-wave pair kernel (libmuz_convpair1): every root path's GPU tests, root kernel traces, the root microbenchmark A/B.
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
export TMPDIR=/tmp
V=exploring-muzero-on-dog_amd/variants
NEW=exploring-muzero-on-dog_amd/libmuz.so
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_nets.py \
  tests/test_gpu_dog_muzero.py tests/test_gpu_selfplay.py tests/test_gpu_stochastic.py tests/test_gpu_headline.py \
  tests/test_gpu_selfplay_classic.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in $V/libmuz_convpair1.so $NEW; do
  t=$(basename $lib .so)
  MUZ_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/root_$t -o run --output-format csv -- \
    python3 profiles/root_microbench.py 4096 > $O/root_$t.log 2>&1 || { tail -20 $O/root_$t.log; exit 1; }
  find $O/root_$t -name '*kernel_stats.csv' -exec cp {} $O/root_kernel_stats_$t.csv \;
  find $O/root_$t -name '*_kernel_trace.csv' -delete
done
python3 - <<'PY'
import csv
for t in ("libmuz_convpair1", "libmuz"):
    for r in csv.DictReader(open(f"gpurun_out/r6z/root_kernel_stats_{t}.csv")):
        if "film" not in r["Name"]:
            print(t, r["Name"][:30], round(float(r["AverageNs"]) / 1e3, 1))
PY
for rep in 1 2 3; do
  for lib in $V/libmuz_convpair1.so $NEW; do
    MUZ_LIB=$lib timeout -k 10 120 python3 profiles/root_microbench.py 4096 2>&1 | grep root_inference >> $O/root_ab.log || exit 1
  done
done
cat $O/root_ab.log
echo r6z-done
