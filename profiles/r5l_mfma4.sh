#!/bin/bash
# Round 5 (VERDICT r4 item 6, and the 8-row tiles of items 3 / 7): the weight-stream MFMA loop on 16x16x4 (loop_bench)
# against 4x4x1_16b row blocks (loop_bench_4x4: 16 rows with one or two trunks, 8 rows), and the classic search's
# measured branch histogram (diag_classic_branches.py).
set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
B=profiles/_bin
for rep in 1 2; do
  timeout -k 10 60 $B/lb16 || exit 1
  for v in r16_t1_d8 r16_t1_d16 r16_t2_d8 r8_t1_d8 r8_t1_d16 r8_t2_d8; do timeout -k 10 60 $B/lb4_$v || exit 1; done
done 2>&1 | tee $O/mfma4.log
MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_br.so timeout -k 10 300 python3 profiles/diag_classic_branches.py > $O/classic_branches.log 2>&1 || { tail $O/classic_branches.log; exit 1; }
cat $O/classic_branches.log
