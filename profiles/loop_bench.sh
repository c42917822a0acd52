#!/bin/bash
# Runs every built loop_bench variant (exploring-muzero-on-dog_amd/variants/lb/lb_*) at 256 workgroups (all
# CUs, L2 shared) and at 1 workgroup (one CU alone); output in gpurun_out/loop_bench.log
set -o pipefail
mkdir -p gpurun_out
for g in 256 1; do
  for b in exploring-muzero-on-dog_amd/variants/lb/lb_*; do
    echo -n "grid $g $(basename $b): " >> gpurun_out/loop_bench.log
    timeout -k 5 60 $b $g 40 >> gpurun_out/loop_bench.log 2>&1 || exit 1
  done
done
cat gpurun_out/loop_bench.log
