#!/bin/bash
# Round 4 verdict item 7: HBM bytes of the env round kernel at 2^20 games (k_det_round) by PMC, FETCH_SIZE and
# WRITE_SIZE in separate passes, then the bench line (which reads the committed summary).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
B=1048576
timeout -k 10 600 python -u -m pytest tests/test_gpu_env_round.py -x -q --timeout 300 --timeout-method thread > $O/env_tests.log 2>&1 \
  || { tail -30 $O/env_tests.log; exit 1; }
tail -1 $O/env_tests.log
for rep in 1 2; do
  for v in r3 new; do
    if [ $v = new ]; then unset MUZ_LIB; else export MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_$v.so; fi
    timeout -k 10 300 python3 bench.py --workload env --batch $B --steps 5 --warmup 1 --no-cpu-baseline > $O/ab_$v$rep.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/ab_$v$rep.json')); print('$v', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
unset MUZ_LIB
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $P --kernel-include-regex "k_det_round" -d $O/p_$P -o run --output-format csv -- \
    python3 bench.py --workload env --batch $B --steps 2 --warmup 1 --no-cpu-baseline > $O/p_$P.log 2>&1 || { tail -20 $O/p_$P.log; exit 1; }
done
python3 profiles/summarize_env_pmc.py $O $B > $O/env_pmc_$B.json && cat $O/env_pmc_$B.json
timeout -k 10 300 python3 bench.py --workload env --batch $B --steps 5 --warmup 1 > $O/env_bench_$B.json 2> $O/env_bench.err || { tail $O/env_bench.err; exit 1; }
cut -c1-600 $O/env_bench_$B.json
