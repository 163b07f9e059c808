#!/bin/bash
# Focused PMC passes on the acquisition correlate kernel (C2 workload, 64 blocks).
# Usage: profiles/collect_acq.sh OUTDIR [variant]
set -o pipefail
OUT=${1:-gpurun_out/pmc_acq}
export GSDR_ACQ_CORR_VARIANT=${2:-0}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
      python3 profiles/acq_driver.py --iters 2 --what acq > "$OUT/$name.log" 2>&1 || return 1
}
run a SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU &&
run b SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL &&
run c SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE SQ_CYCLES &&
run d TCC_HIT_sum TCC_MISS_sum
echo "collect exit $?"
