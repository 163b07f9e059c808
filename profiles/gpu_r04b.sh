#!/bin/bash
# r04b: phase ablations of the wave-local split correlate (ids 112/212, 113/213:
# without phase 1's loads / without phase 2) under rocprofv3 kernel traces, for
# the C4 4 ms (N = 32000) and bit-transition (N = 64000) acquisitions.
#   gpurun --timeout 900 -- bash profiles/gpu_r04b.sh TAG
set -o pipefail
TAG=${1:-r04b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "C4s 2" "C4s 12" "C4s 112" "C4s 212" "C4 3" "C4 13" "C4 113" "C4 213"; do
  set -- $spec
  echo "== $1 split id $2"
  GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$1_$2" -o run \
      -- python3 profiles/acq_cfg_driver.py --cfg $1 --iters 4 > "$OUT/log_$1_$2.txt" 2>&1 || { tail -5 "$OUT/log_$1_$2.txt"; exit 1; }
  f=$(find "$OUT/prof_$1_$2" -name "*kernel_stats.csv" | head -1)
  grep -E "split|forward|argmax|second" "$f" | cut -d, -f1-5 | sed 's/acq_correlate_split_kernel/SPLIT/' | cut -c1-200
done
