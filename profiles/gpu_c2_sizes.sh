#!/bin/bash
# C2 bench (20/5) with the acquisition chains' block counts given per spec ("64" = one chain,
# "32,32", "40,24", ...), each run twice, alternating.
set -o pipefail
OUT=gpurun_out/sizes
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for S in "$@"; do
    n=${S//,/_}
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --acq-sizes $S \
        > "$OUT/c2_${n}_$rep.json" 2> "$OUT/c2_${n}_$rep.err" || exit $?
    python3 -c "
import json
d=json.loads(open('$OUT/c2_${n}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$S rep $rep', d['value'], 'corr', r['avg_launch_us'], 'busy', r['busy_us_per_step'], 'acq_only', d['components']['acq_only_msps'], d['check']['channels_within_25hz'])
"
  done
done
