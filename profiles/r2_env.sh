#!/bin/bash
# Env-only micro-benchmark (SURVEY 8(d)(b')): parity tests of the fused round kernel, bench lines at the
# config batch (4096) and at an HBM-sized batch (2^20 games), and a kernel-trace summary of the large one.
set -o pipefail
O=gpurun_out/r2_env
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_env_round.py -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 200 python bench.py --workload env --steps 5 --warmup 1 --cpu-seconds 10 > $O/bench_4096.json 2> $O/bench_4096.err || { tail -20 $O/bench_4096.err; exit 1; }
timeout -k 10 200 python bench.py --workload env --batch 1048576 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_1m.json 2> $O/bench_1m.err || { tail -20 $O/bench_1m.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --workload env --batch 1048576 --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
cat $O/bench_4096.json $O/bench_1m.json
