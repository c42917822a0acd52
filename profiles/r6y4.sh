#!/bin/bash
# Round 6 end, final HEAD (Dense_0 k split): learner steps (with / without the loss handout), smoke, the whole GPU suite, the default bench line
# (headline) and its kernel trace.
set -o pipefail
O=gpurun_out/r6y4
mkdir -p $O
export TMPDIR=/tmp
for game in det dog; do
  timeout -k 10 300 python3 profiles/r5_learner_steps.py 30 $game 2>&1 | grep "ms per step" >> $O/steps.log || exit 1
done
cat $O/steps.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/trace -name '*_kernel_trace.csv' -delete
head -7 $O/kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
echo r6y-done
