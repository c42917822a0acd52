#!/bin/bash
# Round 6: DOG search with the visited records' cached exp(prior - max prior): the DOG search / records GPU tests
# (bit-identical to the restatement), the DOG MuZero bench A/B against the build before it (2 interleaved reps),
# and the stamp build's cycle shares.
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_dog_muzero.py \
  tests/test_gpu_dog_records.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$PWD/exploring-muzero-on-dog_amd/variants
for rep in 1 2; do
  for v in r6c new; do
    if [ $v = new ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 300 python3 bench.py --workload dog --policy muzero --steps 4 --warmup 1 --no-cpu-baseline > $O/dog_${v}_$rep.json 2> $O/dog_${v}_$rep.err || { tail -20 $O/dog_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/dog_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', $rep, d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
unset MUZ_LIB
MUZ_LIB=$V/libmuz_st2.so timeout -k 10 300 python profiles/diag_dog_stamps.py selfplay > $O/dog_stamps_selfplay.log 2>&1 || { tail -20 $O/dog_stamps_selfplay.log; exit 1; }
cat $O/dog_stamps_selfplay.log
echo r6f-done
