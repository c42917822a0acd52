#!/bin/bash
# Round 6: the DOG evaluation harness tests; k_repr_conv A/B (round-6 base build = round-5 conv, the unpadded-rows
# build, the default) by kernel trace; the DOG search cycle shares on the visited-mask tree (stamp build).
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_evaluate_dog.py \
  > $O/eval_dog_tests.log 2>&1 || { tail -30 $O/eval_dog_tests.log; exit 1; }
tail -2 $O/eval_dog_tests.log
V=$PWD/exploring-muzero-on-dog_amd/variants
for rep in 1 2; do
  for v in r6base convpad0 default; do
    if [ $v = default ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/conv_${v}_$rep -o run --output-format csv -- \
      python3 profiles/root_microbench.py 4096 > $O/conv_${v}_$rep.log 2>&1 || { tail -20 $O/conv_${v}_$rep.log; exit 1; }
    find $O/conv_${v}_$rep -name '*_kernel_trace.csv' -delete
  done
done
unset MUZ_LIB
MUZ_LIB=$V/libmuz_st2.so timeout -k 10 300 python profiles/diag_dog_stamps.py selfplay > $O/dog_stamps_selfplay.log 2>&1 || { tail -20 $O/dog_stamps_selfplay.log; exit 1; }
cat $O/dog_stamps_selfplay.log
echo r6e-done
