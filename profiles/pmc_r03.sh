#!/bin/bash
# PMC passes of HEAD's kernels (MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and
# WRITE_SIZE in separate passes, --kernel-trace --stats --pmc only, one counter group
# per run), each under its own time limit:
#  - C2, the bench workload: profiles/acq_driver.py --what acq (forward, correlate,
#    argmax as the bench launches them) and --what trk (the 8-channel trk_kernel);
#  - C4, bit-transition acquisition (FFT 64000 on the default split correlate):
#    profiles/acq_cfg_driver.py --cfg C4.
# Summaries: $OUT/pmc.json (C2, read by bench.py as the roofline "traffic" when
# copied to profiles/pmc_<tag>.json) and $OUT/pmc_c4.json.
#   gpurun -- bash profiles/pmc_r03.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmc_r03}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc "$@" -d "$OUT/c2/$name" -o run --output-format csv -- \
      python3 profiles/acq_driver.py --iters 2 --what acq > "$OUT/c2_$name.log" 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc "$@" -d "$OUT/c2/trk_$name" -o run --output-format csv -- \
      python3 profiles/acq_driver.py --iters 2 --what trk > "$OUT/c2_trk_$name.log" 2>&1 || return 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc "$@" -d "$OUT/c4/$name" -o run --output-format csv -- \
      python3 profiles/acq_cfg_driver.py --cfg C4 --iters 2 > "$OUT/c4_$name.log" 2>&1 || return 1
}
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES &&
run sqb SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE &&
run l2 TCC_HIT_sum TCC_MISS_sum &&
python3 profiles/pmc_summary.py --json "$OUT/c2" > "$OUT/pmc.json" &&
python3 profiles/pmc_summary.py --cfg-json "$OUT/c4" > "$OUT/pmc_c4.json" && cat "$OUT/pmc_c4.json"
rc=$?
echo "pmc exit $rc"
exit $rc
