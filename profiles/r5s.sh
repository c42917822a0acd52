#!/bin/bash
# Round 5: HEAD check -- full GPU suite (lean DOG checks, AdamW device table, conv LDS aliasing, learner folds), smoke,
# headline bench + rocprofv3 kernel stats; then k_dog_play lean-check A/B (stamps + bench, 2 interleaved reps) and
# the learner step trace.
set -o pipefail
O=gpurun_out/r5s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
cp gpurun_out/parity.log $O/parity.log 2>/dev/null
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name '*_kernel_trace.csv' -delete
head -8 $O/kernel_stats.csv | cut -c1-160
V=$PWD/exploring-muzero-on-dog_amd/variants
MUZ_LIB=$V/libmuz_dogst.so timeout -k 10 120 python3 profiles/diag_dog_play_stamps.py > $O/dog_stamps_lean.log 2>&1 || { tail $O/dog_stamps_lean.log; exit 1; }
cat $O/dog_stamps_lean.log
for rep in 1 2; do
  for v in nolean lean; do
    if [ $v = lean ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 300 python3 bench.py --workload dog --steps 5 --warmup 1 --no-cpu-baseline > $O/dog_$v$rep.json 2> $O/dog_$v$rep.err || { tail $O/dog_$v$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/dog_$v$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline'].get('achieved'), d['roofline'].get('frac'))"
  done
done
unset MUZ_LIB
bash profiles/r5_learner_trace.sh r5s det > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
head -12 gpurun_out/prof_learner_r5s/step_per_kernel.txt
