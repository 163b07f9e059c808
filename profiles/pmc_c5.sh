#!/bin/bash
# PMC passes of the C5 acquisition grids on HEAD (GPS N = 25000: C5g, Galileo N = 100000: C5e),
# one counter group per run, --kernel-trace --stats --pmc only, each under its own limit.
#   gpurun -- bash profiles/pmc_c5.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmc_c5}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  for cfg in C5e C5g; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc "$@" -d "$OUT/$cfg/$name" -o run --output-format csv -- \
        python3 profiles/acq_cfg_driver.py --cfg $cfg --iters 2 > "$OUT/${cfg}_$name.log" 2>&1 || return 1
  done
}
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES &&
run sqb SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE &&
run l2 TCC_HIT_sum TCC_MISS_sum &&
python3 profiles/pmc_summary.py --cfg-json "$OUT/C5e" > "$OUT/pmc_c5e.json" &&
python3 profiles/pmc_summary.py --cfg-json "$OUT/C5g" > "$OUT/pmc_c5g.json" && cat "$OUT/pmc_c5e.json"
rc=$?
echo "pmc exit $rc"
exit $rc
