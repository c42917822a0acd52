#!/bin/bash
# Round 4: rocprofv3 kernel stats of the DOG MuZero bench line (k_dog_search's average launch against the line's
# avg_launch_ms).
set -o pipefail
O=gpurun_out/r4zf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --workload dog --policy muzero --steps 2 --warmup 1 --no-cpu-baseline > $O/dog_mz_prof.json 2> $O/dog_mz_prof.err || { tail -20 $O/dog_mz_prof.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name '*_kernel_trace.csv' -delete
head -8 $O/kernel_stats.csv | cut -c1-200
cut -c1-200 $O/dog_mz_prof.json
