#!/bin/bash
# A/B of the last-stage block padding (variant 81 = 70 + PADL 9) in the C2 bench, interleaved.
set -o pipefail
O=gpurun_out/padl2; mkdir -p $O
for i in 1 2 3; do
  for v in 70 81; do
    GSDR_ACQ_CORR_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b${v}_$i.json 2> $O/b${v}_$i.err || exit 1
  done
done
timeout -k 10 300 python -u profiles/sweep_acq_n.py --fs 4000000 --blocks 64 --reps 60 --variants 70,81,70,81,70,81 > $O/sweep.jsonl 2>/dev/null
python3 - <<'P'
import json,glob
for f in sorted(glob.glob("gpurun_out/padl2/b*.json")):
    d=json.load(open(f)); print(f.split("/")[-1], d["value"], d["stages_us_per_launch"]["acq_forward"], d["stages_us_per_launch"]["acq_correlate"])
P
cat $O/sweep.jsonl
