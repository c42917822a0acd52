#!/bin/bash
# Round 5: k_dog_search PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and kernel trace at the round's
# default launch (6 games per workgroup at 1500 games).
set -o pipefail
O=gpurun_out/r5zd
mkdir -p $O
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_dog_search -d $O/dog_pmc_$C -o run --output-format csv -- \
    python3 bench.py --workload dog --policy muzero --steps 1 --warmup 0 --no-cpu-baseline > $O/dog_pmc_$C.log 2>&1 || { tail -20 $O/dog_pmc_$C.log; exit 1; }
done
python3 profiles/summarize_pmc_kernel.py $O/dog_pmc_FETCH_SIZE $O/dog_pmc_WRITE_SIZE k_dog_search "profiles/r5zd.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-include-regex k_dog_search, separate passes of bench.py --workload dog --policy muzero --steps 1 --warmup 0; 6 games per workgroup)" > $O/dog_traffic.json || exit 1
cat $O/dog_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dog_trace -o run --output-format csv -- \
  python3 bench.py --workload dog --policy muzero --steps 1 --warmup 1 --no-cpu-baseline > $O/dog_trace.log 2>&1 || { tail -20 $O/dog_trace.log; exit 1; }
find $O/dog_trace -name '*kernel_stats.csv' -exec cp {} $O/dog_kernel_stats.csv \;
find $O/dog_trace -name '*_kernel_trace.csv' -delete
head -4 $O/dog_kernel_stats.csv | cut -c1-150
