#!/bin/bash
# Round 4, first check on a MI355X: exact tree arithmetic (search.hip: no contraction, numpy-order sums,
# correctly rounded exp) -- parity tests with the >1e-5 counts, smoke, A/B vs the round-3 build, timeline.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
rm -f gpurun_out/parity.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_headline.py tests/test_gpu_selfplay.py \
  tests/test_gpu_reference_api.py tests/test_gpu_nets.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
cp gpurun_out/parity.log $O/parity.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
V=exploring-muzero-on-dog_amd/variants
for rep in 1 2 3; do
  for v in r3 new; do
    if [ $v = new ]; then unset MUZ_LIB; else export MUZ_LIB=$PWD/$V/libmuz_$v.so; fi
    timeout -k 10 120 python3 profiles/search_microbench.py 4096 50 2>/dev/null | tee -a $O/ab.log || exit 1
  done
done
unset MUZ_LIB
MUZ_LIB=$PWD/$V/libmuz_tl.so timeout -k 10 120 python3 profiles/diag_timeline.py 4096 > $O/timeline.log 2>&1 || { tail -20 $O/timeline.log; exit 1; }
tail -25 $O/timeline.log
