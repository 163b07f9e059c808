#!/bin/bash
# SQ counters of the correlate kernel for several GSDR_ACQ_CORR_VARIANT values.
#   gpurun -- bash profiles/pmc_variants.sh TAG v1,v2,...
set -o pipefail
OUT=gpurun_out/${1:-pmcv}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $(echo ${2:-35,42} | tr , ' '); do
  export GSDR_ACQ_CORR_VARIANT=$v
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES \
     -d "$OUT/v$v/a" -o run --output-format csv -- python3 profiles/acq_driver.py --iters 2 --what acq > "$OUT/v$v.log" 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
     -d "$OUT/v$v/b" -o run --output-format csv -- python3 profiles/acq_driver.py --iters 2 --what acq >> "$OUT/v$v.log" 2>&1 || exit 1
  echo "== variant $v"; python3 profiles/pmc_summary.py "$OUT/v$v" correlate
done
