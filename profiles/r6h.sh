#!/bin/bash
# Round 6: DOG search stamp shares at two batch sizes (the self-play setting): 1500 games (250 workgroups) and 256
# (43): a smaller tree / fewer workgroups per XCD L2 -- how much of a walk level is memory latency.
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
V=$PWD/exploring-muzero-on-dog_amd/variants
for b in 1500 256; do
  DIAG_B=$b MUZ_LIB=$V/libmuz_st2.so timeout -k 10 300 python profiles/diag_dog_stamps.py selfplay > $O/dog_stamps_$b.log 2>&1 || { tail -20 $O/dog_stamps_$b.log; exit 1; }
  cat $O/dog_stamps_$b.log
done
echo r6h-done
