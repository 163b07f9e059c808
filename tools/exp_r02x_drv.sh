#!/bin/bash
# The driver's bench flags (--steps 20 --warmup 5): default vs no profiling events vs 4 chains.
set -o pipefail
O=gpurun_out/drv2; mkdir -p $O
for i in 1 2; do
  for cfg in "def:" "noev:--no-profile-events" "ch4:--acq-chains 4" "ch1:--acq-chains 1"; do
    tag=${cfg%%:*}; opts=${cfg#*:}
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $opts > $O/${tag}_$i.json 2> $O/${tag}_$i.err || exit 1
  done
done
python3 - <<'P'
import json,glob
for f in sorted(glob.glob("gpurun_out/drv2/*.json")):
    d=json.load(open(f)); print(f.split("/")[-1], d["value"], d["ms_per_step"], d.get("stages_us_per_launch",{}).get("acq_correlate"), d["check"]["channels_within_25hz"])
P
