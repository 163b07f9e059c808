#!/bin/bash
# PMC passes (MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE / WRITE_SIZE in separate
# passes, --kernel-trace --pmc only, one counter group per run) over
#  - the C2 bench workload: profiles/acq_driver.py --what acq (acquisition forward,
#    correlate and argmax kernels, as the bench launches them) and --what trk (the
#    8-channel trk_kernel), and
#  - the C3 multicorrelator epochs (profiles/configs_bench.py --only C3: corr_kernel).
# Summarised to $OUT/pmc.json by profiles/pmc_summary.py --json.
#   gpurun -- bash profiles/pmc_round2.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
      python3 profiles/acq_driver.py --iters 2 --what acq > "$OUT/$name.log" 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/trk_$name" -o run --output-format csv -- \
      python3 profiles/acq_driver.py --iters 2 --what trk > "$OUT/trk_$name.log" 2>&1 || return 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/c3_$name" -o run --output-format csv -- \
      python3 profiles/configs_bench.py --only C3 --reps 2 > "$OUT/c3_$name.log" 2>&1 || return 1
}
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES &&
run sqb SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE &&
run l2 TCC_HIT_sum TCC_MISS_sum &&
python3 profiles/pmc_summary.py --json "$OUT" > "$OUT/pmc.json" && cat "$OUT/pmc.json"
echo "pmc exit $?"
