#!/bin/bash
# Round 5: how much of k_root_dense is Dense_0 (3584 -> 256): root_inference microbenchmark at 4096 games with the
# in-tree build and a timing-only build that leaves Dense_0 out (-DMUZ_EXPT_SKIP_D0, wrong results), 3 interleaved reps.
set -o pipefail
O=gpurun_out/r5zf
mkdir -p $O
V=$PWD/exploring-muzero-on-dog_amd/variants
for rep in 1 2 3; do
  for v in base skipd0; do
    if [ $v = base ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 120 python3 profiles/root_microbench.py 4096 2>&1 | grep root_inference || exit 1
  done
done
