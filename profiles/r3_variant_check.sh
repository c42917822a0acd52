#!/bin/bash
# A/B of a k_gumbel_search variant (exploring-muzero-on-dog_amd/variants/libmuz_<v>.so) against the in-tree
# libmuz.so, then the variant's net / search parity tests:  bash profiles/r3_variant_check.sh <v> [pytest files]
set -o pipefail
V=$1
shift
O=gpurun_out/var_$V
mkdir -p $O
VL=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_$V.so
for rep in 1 2 3; do
  for lib in base $V; do
    if [ $lib = base ]; then unset MUZ_LIB; else export MUZ_LIB=$VL; fi
    timeout -k 10 120 python3 profiles/search_microbench.py 4096 50 2>/dev/null | tee -a $O/ab.log || exit 1
  done
done
unset MUZ_LIB
TESTS=${@:-tests/test_gpu_nets.py tests/test_gpu_search.py tests/test_gpu_headline.py}
MUZ_LIB=$VL timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
