# PMC passes over the env-only round kernel (k_det_round) at 2^20 games (bench.py --workload env): instruction
# mix, issue / LDS utilisation and HBM bytes, to place it against its bounds.  One rocprofv3 --pmc pass per
# counter set; per-launch means -> gpurun_out/prof_env_pmc/summary.json (profiles/summarize_env_pmc.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_env_pmc
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
P5="GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $P --kernel-include-regex k_det_round -d $O/p$i -o run --output-format csv -- python3 bench.py --workload env --batch 1048576 --steps 2 --warmup 1 --no-cpu-baseline > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python3 profiles/summarize_env_pmc.py $O > $O/summary.json && cat $O/summary.json
