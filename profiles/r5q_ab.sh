#!/bin/bash
# Round 5, VERDICT r4 item 5 Option A: search microbenchmark A/B, dense16 + ln16 (in-tree libmuz.so, MUZ_LN_EPILOGUE=0)
# against dense_ln16 (libmuz_lne.so, MUZ_LN_EPILOGUE=1), B=4096 S=50, 4 interleaved repetitions.
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
V=$PWD/exploring-muzero-on-dog_amd/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner_fused.py -x -q -k "film" --timeout 200 --timeout-method thread > $O/film_tests.log 2>&1 || { tail -40 $O/film_tests.log; exit 1; }
tail -1 $O/film_tests.log
bash profiles/r5_learner_trace.sh r5q det > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
grep -E "film|one train" gpurun_out/prof_learner_r5q/step_per_kernel.txt
for rep in 1 2 3 4; do
  for v in off lne; do
    if [ $v = off ]; then unset MUZ_LIB; else export MUZ_LIB=$V/libmuz_$v.so; fi
    timeout -k 10 120 python3 profiles/search_microbench.py 4096 50 2>/dev/null | sed "s/^/$v /" | tee -a $O/ab.log || exit 1
  done
done
# learner: the grouped weight-gradient launch with 512 / 1024-row segments (MUZ_WGRAD_SEG) against 2048
for seg in 512 1024; do
  MUZ_LIB=$V/libmuz_seg$seg.so bash profiles/r5_learner_trace.sh r5q_seg$seg det > $O/trace_seg$seg.log 2>&1 || { tail $O/trace_seg$seg.log; exit 1; }
  echo "seg $seg:"; grep -E "k_wgrad|k_colsum|one train" gpurun_out/prof_learner_r5q_seg$seg/step_per_kernel.txt
done
