# PMC passes over the DOG actor kernel (config d bench, 1024 games, 16 turns per launch): instruction mix
# and issue utilisation, to place k_dog_play against the VALU issue rate.  Summary: profiles/summarize_pmc.py
# style means per launch -> profiles/<tag>_dog_pmc.json (python profiles/summarize_dog_pmc.py <tag>).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_${1:-r1}_dog_pmc
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVES"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex k_dog_play -d $O/p$i -o run --output-format csv -- python3 bench.py --workload dog --steps 40 --warmup 2 --no-cpu-baseline > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
echo done
