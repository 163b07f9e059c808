#!/bin/bash
# SQ counters of the tracking kernel in the C5 pool (12 GPS + 12 Galileo + 8 BeiDou,
# three streams): two counter passes, --kernel-trace --stats --pmc only.
#   gpurun -- bash profiles/pmc_trk.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmc_trk}
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
      python3 profiles/configs_bench.py --only C5 --reps 1 > "$OUT/$name.log" 2>&1
}
pass p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    SQ_INSTS_VALU SQ_INSTS_LDS &&
pass p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CYCLES \
    SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC &&
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "trk_kernel" not in r.get("Kernel_Name", ""): continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot): print(f"{k:24s} {tot[k]:16.0f}  ({n[k]} rows)")
PY
