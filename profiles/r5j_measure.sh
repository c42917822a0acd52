#!/bin/bash
# Round-5 measurements of the other workloads on HEAD:
#   config (c) classic bench + rocprofv3 kernel trace;  DOG MuZero bench + FETCH_SIZE / WRITE_SIZE passes on
#   k_dog_search;  the det learner step trace (train_step_from);  the DOG train loop with --overlap.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 400 python3 bench.py --workload classic --steps 2 --warmup 1 > $O/classic.json 2> $O/classic.err || { tail -20 $O/classic.err; exit 1; }
tail -1 $O/classic.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/classic_trace -o run --output-format csv -- \
  python3 bench.py --workload classic --steps 1 --warmup 1 --no-cpu-baseline > $O/classic_trace.log 2>&1 || { tail -20 $O/classic_trace.log; exit 1; }
timeout -k 10 300 python3 bench.py --workload dog --policy muzero > $O/dog_mz.json 2> $O/dog_mz.err || { tail -20 $O/dog_mz.err; exit 1; }
tail -1 $O/dog_mz.json | cut -c1-400
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex k_dog_search -d $O/dog_pmc_$C -o run --output-format csv -- \
    python3 bench.py --workload dog --policy muzero --steps 1 --warmup 0 --no-cpu-baseline > $O/dog_pmc_$C.log 2>&1 || { tail -20 $O/dog_pmc_$C.log; exit 1; }
done
bash profiles/r5_learner_trace.sh r5j det || exit 1
timeout -k 10 600 python3 bench.py --workload train --game dog --overlap --steps 2 --warmup 1 > $O/train_dog_overlap.json 2> $O/train_dog_overlap.err || { tail -20 $O/train_dog_overlap.err; exit 1; }
tail -1 $O/train_dog_overlap.json | cut -c1-400
echo measure-done
