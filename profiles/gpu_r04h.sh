#!/bin/bash
# r04h: kernel traces of the large-N acquisitions with the forward-spectrum reuse,
# incl. the phase ablations of the split correlate (ids 1xx: no phase-1 loads, 2xx:
# no phase 2).  Spec "cfg|ENV=.." per run.
#   gpurun --timeout 900 -- bash profiles/gpu_r04h.sh TAG "C4|" "C4|GSDR_ACQ_SPLIT_ID=113" ...
set -o pipefail
TAG=${1:-r04h}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for SPEC in "$@"; do
  IFS='|' read -r cfg ENVS <<< "$SPEC"
  i=$((i+1)); name="${cfg}_$i"
  echo "== $cfg $ENVS"
  env GSDR_ACQ_SPLIT=2 $ENVS timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$name" -o run \
      --output-format csv -- python3 profiles/acq_cfg_driver.py --cfg $cfg --iters 4 > "$OUT/log_$name.txt" 2>&1 \
      || { tail -5 "$OUT/log_$name.txt"; exit 1; }
  f=$(find "$OUT/prof_$name" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$OUT/stats_$name.csv"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "acq_" not in n: continue
    short = n.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[:90]
    print("   %-90s calls %4s avg %9.1f us" % (short, r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
echo "exit 0"
