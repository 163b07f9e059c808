#!/bin/bash
# Co-run cost of tracking in the C2 step on one box: default, CU-partitioned tracking
# (8 / 16 CUs), acquisition alone; each twice, interleaved.
set -o pipefail
O=gpurun_out/corun; mkdir -p $O
for i in 1 2; do
  for cfg in "def:" "part8:--cu-partition" "part16:--cu-partition --trk-cus 16" "acq:--only acq"; do
    tag=${cfg%%:*}; opts=${cfg#*:}
    timeout -k 10 200 python bench.py --no-cpu-baseline $opts > $O/${tag}_$i.json 2> $O/${tag}_$i.err || exit 1
  done
done
python3 - <<'P'
import json,glob
for f in sorted(glob.glob("gpurun_out/corun/*.json")):
    d=json.load(open(f)); print(f.split("/")[-1], d["value"], d["stages_us_per_launch"].get("acq_correlate"), d.get("check",{}).get("channels_within_25hz"))
P
