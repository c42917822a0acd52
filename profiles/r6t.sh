#!/bin/bash
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp
for sk in 1 0; do
  MUZ_SPLITK_DENSE=$sk timeout -k 10 600 python3 -u profiles/diag_splitk.py > $O/diag_sk$sk.log 2>&1 || { tail -30 $O/diag_sk$sk.log; exit 1; }
  echo "== splitk $sk"; grep -v "amdgpu.ids\|^/opt" $O/diag_sk$sk.log
done
echo r6t-done
