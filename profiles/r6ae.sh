#!/bin/bash
# Round 6: rocprofv3 kernel trace of the DOG MuZero bench line on the round-end build (the rocprof basis of its frac),
# then the line itself reading it.
set -o pipefail
O=gpurun_out/r6ae
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --workload dog --policy muzero --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/dog_kernel_stats.csv \;
find $O/trace -name '*_kernel_trace.csv' -delete
cp $O/dog_kernel_stats.csv profiles/r6ae_dog_kernel_stats.csv
head -3 $O/dog_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
timeout -k 10 400 python3 bench.py --workload dog --policy muzero --steps 3 --warmup 1 --no-cpu-baseline > $O/dog_mz.json 2> $O/dog_mz.err || { tail -20 $O/dog_mz.err; exit 1; }
tail -1 $O/dog_mz.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['frac'], r['avg_launch_ms'], r['frac_rocprof'], r['rocprof_avg_launch_ms'])"
echo r6ae-done
