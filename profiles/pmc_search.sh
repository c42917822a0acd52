set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_${1:-r1}_pmc
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
P4="TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex k_gumbel_search -d $O/p$i -o run --output-format csv -- python3 profiles/search_microbench.py 4096 50 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
echo done
