#!/bin/bash
# Round 4: learner step kernel trace at HEAD (ResBlock stack kernels) + config (e) iteration, sequential and overlapped.
set -o pipefail
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 400 bash profiles/r3_learner_trace.sh r4n > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cat $O/trace.log
cp gpurun_out/prof_learner_r3_r4n/step_per_kernel.txt $O/ 2>/dev/null
cp gpurun_out/prof_learner_r3_r4n/step_sequence.txt $O/ 2>/dev/null
timeout -k 10 400 python bench.py --workload train --steps 1 --warmup 1 > $O/train.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
cut -c1-300 $O/train.json
timeout -k 10 500 python bench.py --workload train --overlap --steps 2 --warmup 1 > $O/train_overlap.json 2> $O/train_overlap.err || { tail -20 $O/train_overlap.err; exit 1; }
cut -c1-300 $O/train_overlap.json
