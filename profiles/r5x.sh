#!/bin/bash
# Round 5: the det turn head as one launch (k_sp_head: refill + flags + compaction + encode, decoupled look-back
# scans) -- self-play / headline GPU tests, then an interleaved headline A/B against the four-launch head
# (variants/libmuz_nohead.so), and a kernel trace of the fused build.
set -o pipefail
O=gpurun_out/${R5X_OUT:-r5x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_headline.py tests/test_gpu_reference_api.py tests/test_gpu_replay.py tests/test_gpu_evaluate.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$PWD/exploring-muzero-on-dog_amd/variants
for rep in 1 2; do
  for v in nohead head; do
    if [ $v = head ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/b_$v$rep.json 2> $O/b_$v$rep.err || { tail $O/b_$v$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_$v$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['end_to_end_frac'])"
  done
done
unset MUZ_LIB
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name '*_kernel_trace.csv' -delete
head -12 $O/kernel_stats.csv | cut -c1-120
