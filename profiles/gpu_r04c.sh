#!/bin/bash
# r04c: SQ counters of the wave-local split correlate (C4 4 ms id 12, C4 bit
# transition id 13) and of the round-3 default (ids 2, 3): one counter group per
# rocprofv3 run, --kernel-trace --pmc only.
#   gpurun --timeout 900 -- bash profiles/gpu_r04c.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r04c}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local cfg=$1 id=$2 name=$3; shift 3
  GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=$id timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" \
      -d "$OUT/${cfg}_${id}/$name" -o run --output-format csv -- \
      python3 profiles/acq_cfg_driver.py --cfg $cfg --iters 2 > "$OUT/${cfg}_${id}_$name.log" 2>&1
}
for spec in "C4s 12" "C4 13" "C4s 2" "C4 3"; do
  set -- $spec
  run $1 $2 sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES &&
  run $1 $2 sqb SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit 1
  echo "== $1 $2"; python3 profiles/pmc_summary.py "$OUT/${1}_${2}" split
done
