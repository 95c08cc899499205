#!/bin/bash
# Bottleneck PMC passes (memory pipeline, LDS, issue) over tools/prof_kernels.py, one rocprofv3
# run per counter group; never combined with tracing. Usage: tools/pmc2.sh <outdir> [config]
out=${1:-gpurun_out/pmc2}; cfg=${2:-c3}
export TMPDIR=/tmp
mkdir -p "$out"
groups=(
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL"
  "TD_TD_BUSY_sum TD_TC_STALL_sum TCC_BUSY_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_LEVEL_sum"
  "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUSY_max"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA"
  "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS"
)
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 60 rocprofv3 --pmc $g --output-format csv -d "$out/p$i" -o run -- python3 tools/prof_kernels.py --config $cfg --reps 10 > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after rc=$rc"; exit $rc;; esac
done
python3 tools/pmc_summary.py "$out"
