#!/bin/bash
# Round-5 refresh of the headline's measured ceilings on HEAD: the loop bench, the headline bench +
# rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (profile_bench.sh), and the search PMC passes
# (pmc_search.sh: TCP_TCC_READ_REQ, SQ_VALU_MFMA_BUSY_CYCLES, ...).  Summaries: summarize_profile.py / summarize_pmc.py r5i.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/loop_bench.log
for g in 256 1; do
  echo -n "grid $g lb_base: " >> gpurun_out/loop_bench.log
  timeout -k 5 60 exploring-muzero-on-dog_amd/variants/lb/lb_base $g 40 >> gpurun_out/loop_bench.log 2>&1 || exit 1
done
cp gpurun_out/loop_bench.log gpurun_out/r5i_loop_bench.log
bash profiles/profile_bench.sh r5i || exit 1
bash profiles/pmc_search.sh r5i || exit 1
echo measure-done
