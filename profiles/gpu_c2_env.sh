#!/bin/bash
# C2 bench (20/5) A/B over env specs "name|ENV=.. ENV=..", twice, interleaved.
#   gpurun --timeout 900 -- bash profiles/gpu_c2_env.sh TAG "a|X=1" "b|X=2"
set -o pipefail
TAG=${1:-c2env}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for SPEC in "$@"; do
    IFS='|' read -r name ENVS <<< "$SPEC"
    env $ENVS timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        > "$OUT/c2_${name}_$rep.json" 2> "$OUT/c2_${name}_$rep.err" || exit $?
    python3 -c "
import json
d=json.loads(open('$OUT/c2_${name}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name rep $rep', d['value'], 'corr', r['avg_launch_us'], 'busy', r['busy_us_per_step'], 'frac', r['frac'], 'acq_only', d['components']['acq_only_msps'])
"
  done
done
