#!/bin/bash
# Kernel-trace + PMC passes for the dominant kernels (run on the GPU box from the repo root).
# Counters are collected in separate passes (--pmc only with --kernel-trace), per
# MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass.
set -o pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
      python3 profiles/acq_driver.py --iters 3 > "$OUT/$name.log" 2>&1 || return 1
}
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 profiles/acq_driver.py --iters 10 > "$OUT/trace.log" 2>&1 &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES &&
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE &&
run l2 TCC_HIT_sum TCC_MISS_sum
echo "collect exit $?"
