#!/bin/bash
# C2 bench (driver flags 20/5) A/B, specs "name|ENV=..", each run twice in alternation.
set -o pipefail
TAG=${1:-c2ab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; }
for rep in 1 2; do
for SPEC in "$@"; do
  IFS='|' read -r name ENVS <<< "$SPEC"
  env $ENVS timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c2_${name}_$rep.json" \
      2> "$OUT/c2_${name}_$rep.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  if [ $rc -ne 0 ]; then tail -3 "$OUT/c2_${name}_$rep.err"; exit $rc; fi
  python3 -c "
import json
d=json.loads(open('$OUT/c2_${name}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; s=d['stages_us_per_launch']
print('c2 $name $rep', d['value'], 'corr us', r['avg_launch_us'], 'busy', r['busy_us_per_step'], 'frac', r['frac'], 'fwd', s['acq_forward'], 'reduce', s['acq_reduce'], d['config'].get('forward_spectra_per_block'), d['components'])
"
done
done
