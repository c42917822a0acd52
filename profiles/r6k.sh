#!/bin/bash
# Round 6: the det learner step beside the search (--overlap) -- stream priority A/B, and kernel
# traces of the overlapped and the sequential loop (which learner kernels stretch beside the search).
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
export TMPDIR=/tmp
for p in 0; do
  MUZ_LEARNER_PRIORITY=$p timeout -k 10 400 python3 bench.py --workload train --game det --overlap --steps 2 --warmup 1 \
    > $O/overlap_prio$p.json 2> $O/overlap_prio$p.err || { tail -20 $O/overlap_prio$p.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/overlap_prio$p.json').read().strip().splitlines()[-1]); print('prio $p', d['ms_per_step'], d['roofline']['avg_step_ms'])"
done
for m in overlap seq; do
  flag=""; [ $m = overlap ] && flag="--overlap"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_$m -o run --output-format csv -- \
    python3 bench.py --workload train --game det $flag --steps 1 --warmup 1 > $O/trace_$m.log 2>&1 || { tail -20 $O/trace_$m.log; exit 1; }
  find $O/trace_$m -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_$m.csv \;
  find $O/trace_$m -name '*_kernel_trace.csv' -delete
done
echo r6k-done
