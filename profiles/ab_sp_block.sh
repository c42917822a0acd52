#!/bin/bash
# A/B of the per-lane self-play kernels' workgroup size (k_sp_flags / k_sp_apply, -DMUZ_SP_BLOCK):
#   make -C exploring-muzero-on-dog_amd/csrc BUILD=build_sp64 EXTRA=-DMUZ_SP_BLOCK=64 OUT=../variants/libmuz_sp64.so
#   (same for 128), then through gpurun from the repo root:  bash profiles/ab_sp_block.sh
# Kernel-trace summary per build under gpurun_out/ab_sp/<variant>/, bench lines in gpurun_out/ab_sp/*.json.
set -o pipefail
O=gpurun_out/ab_sp
mkdir -p $O
export TMPDIR=/tmp
for v in 256 64 128; do
  if [ $v = 256 ]; then unset MUZ_LIB; else export MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_sp$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/sp$v -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --games 16384 --no-cpu-baseline > $O/sp$v.json 2> $O/sp$v.err || { tail -20 $O/sp$v.err; exit 1; }
  cat $O/sp$v.json
done
for v in 256 64 128; do
  if [ $v = 256 ]; then unset MUZ_LIB; else export MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/variants/libmuz_sp$v.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_sp$v.json 2> $O/bench_sp$v.err || { tail -20 $O/bench_sp$v.err; exit 1; }
  cat $O/bench_sp$v.json
done
echo ab-done
