#!/bin/bash
# Round 6: the C2 line against the warm-up length (GPU clock ramp?): 20/5 (the driver's flags),
# 20/200, 50/20 (bench.py's defaults), 20/5 again, each a fresh process.
set -o pipefail
TAG=${1:-r06v}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for FL in "--steps 20 --warmup 5" "--steps 20 --warmup 200" "--steps 50 --warmup 20" "--steps 20 --warmup 5" "--steps 200 --warmup 5"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $FL > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/bench_$i.json') if l.startswith('{')][0])
print('$FL |', d['value'], d['ms_per_step'], 'corr us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'], 'acq_only', d['components']['acq_only_msps'])"
  i=$((i + 1))
done
