#!/bin/bash
# r04g: forward-spectrum reuse on the exact carrier (acq_impl.h XMap, gsdr_acq_set_wipeoff):
#  1. the new wipe-off / reuse parity tests, then the whole GPU suite;
#  2. A/B per spec "name|ENV=.. ENV=..": C3/C4/C5 acquisition lines and the C2 bench (20/5).
# A stage that times out or crashes ends the script (no further GPU work).
#   gpurun --timeout 1200 -- bash profiles/gpu_r04g.sh TAG "name|ENV=.." ...
set -o pipefail
TAG=${1:-r04g}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export GSDR_PARITY_LOG=$OUT/parity_spread.jsonl
rm -f "$GSDR_PARITY_LOG"
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; }
echo "== wipe tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_acq_wipe.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_wipe.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_wipe.log"; grep "parity acq_wipe" "$OUT/pytest_wipe.log" | cut -c1-400
if [ $rc -ne 0 ]; then echo "wipe tests rc $rc"; grep -E "Error|assert" "$OUT/pytest_wipe.log" | head -20; exit $rc; fi
echo "== all gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit $rc; fi
for SPEC in "$@"; do
  IFS='|' read -r name ENVS <<< "$SPEC"
  echo "== configs $name ($ENVS)"
  env $ENVS timeout -k 10 240 python -u profiles/configs_bench.py --only C3,C4,C5 --acq-only --reps 6 \
      > "$OUT/cfg_$name.jsonl" 2> "$OUT/cfg_$name.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  python3 -c "
import json
for l in open('$OUT/cfg_$name.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('   ', d['config'], d['stage'][:48], d['msps'], d.get('roofline',{}).get('frac'))
"
  echo "== c2 $name"
  env $ENVS timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c2_$name.json" \
      2> "$OUT/c2_$name.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  python3 -c "
import json
d=json.loads(open('$OUT/c2_$name.json').read().strip().splitlines()[-1]); r=d['roofline']; s=d['stages_us_per_launch']
print('    c2', d['value'], 'corr us', r['avg_launch_us'], 'busy', r['busy_us_per_step'], 'frac', r['frac'], 'fwd', s['acq_forward'], 'reduce', s['acq_reduce'])
"
done
echo "exit 0"
