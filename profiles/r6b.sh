#!/bin/bash
# Round 6: classic evaluation harness tests; PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of
# k_dog_search (visited-mask tree) and k_stochastic_search (config c); TCC_HIT / TCC_MISS of
# k_dog_search (attribute its traffic); kernel-trace stats of both workloads.
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_evaluate_classic.py -k muzero_seats \
  > $O/eval_tests.log 2>&1 || { tail -30 $O/eval_tests.log; exit 1; }
tail -2 $O/eval_tests.log
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  T=$(echo $C | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_dog_search -d $O/dog_pmc_$T -o run --output-format csv -- \
    python3 bench.py --workload dog --policy muzero --steps 1 --warmup 0 --no-cpu-baseline > $O/dog_pmc_$T.log 2>&1 || { tail -20 $O/dog_pmc_$T.log; exit 1; }
done
python3 profiles/summarize_pmc_kernel.py $O/dog_pmc_FETCH_SIZE $O/dog_pmc_WRITE_SIZE k_dog_search "profiles/r6b.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-include-regex k_dog_search, separate passes of bench.py --workload dog --policy muzero --steps 1 --warmup 0; 6 games per workgroup; visited-mask tree)" > $O/dog_traffic.json || exit 1
cat $O/dog_traffic.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_stochastic_search -d $O/classic_pmc_$C -o run --output-format csv -- \
    python3 bench.py --workload classic --steps 1 --warmup 0 --no-cpu-baseline > $O/classic_pmc_$C.log 2>&1 || { tail -20 $O/classic_pmc_$C.log; exit 1; }
done
python3 profiles/summarize_pmc_kernel.py $O/classic_pmc_FETCH_SIZE $O/classic_pmc_WRITE_SIZE k_stochastic_search "profiles/r6b.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-include-regex k_stochastic_search, separate passes of bench.py --workload classic --steps 1 --warmup 0)" > $O/classic_traffic.json || exit 1
cat $O/classic_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dog_trace -o run --output-format csv -- \
  python3 bench.py --workload dog --policy muzero --steps 2 --warmup 1 --no-cpu-baseline > $O/dog_trace.log 2>&1 || { tail -20 $O/dog_trace.log; exit 1; }
find $O/dog_trace -name '*kernel_stats.csv' -exec cp {} $O/dog_kernel_stats.csv \;
find $O/dog_trace -name '*_kernel_trace.csv' -delete
head -4 $O/dog_kernel_stats.csv | cut -c1-150
timeout -k 10 400 python3 bench.py --workload classic --steps 2 --warmup 1 > $O/classic.json 2> $O/classic.err || { tail -20 $O/classic.err; exit 1; }
tail -1 $O/classic.json | cut -c1-300
echo r6b-done
