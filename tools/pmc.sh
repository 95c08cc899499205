#!/bin/bash
# PMC passes over tools/prof_kernels.py (one counter group per rocprofv3 run; --pmc is never
# combined with tracing domains). Usage: tools/pmc.sh <outdir> [config] [prof_kernels args...]
out=${1:-gpurun_out/pmc}; cfg=${2:-c3}; shift $(( $# < 2 ? $# : 2 )); extra="$@"
export TMPDIR=/tmp
mkdir -p "$out"
groups=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32"
)
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $g --output-format csv -d "$out/p$i" -o run -- python3 tools/prof_kernels.py --config $cfg --reps 10 $extra > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc ($g)"
  case $rc in 124|134|137|139) echo "stopping after rc=$rc"; exit $rc;; esac
done
exit 0
