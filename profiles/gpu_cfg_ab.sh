#!/bin/bash
# Acquisition-line A/B: configs_bench --acq-only (C3/C4/C5) per spec "name|ENV=.. ENV=..".
# A stage that times out or crashes ends the script (no further GPU work).
#   gpurun --timeout 900 -- bash profiles/gpu_cfg_ab.sh TAG "name|ENV=.." ...
set -o pipefail
TAG=${1:-cfgab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; }
for SPEC in "$@"; do
  IFS='|' read -r name ENVS <<< "$SPEC"
  echo "== configs $name ($ENVS)"
  env $ENVS timeout -k 10 240 python -u profiles/configs_bench.py --only ${ONLY:-C3,C4,C5} --acq-only --reps 6 \
      > "$OUT/cfg_$name.jsonl" 2> "$OUT/cfg_$name.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  if [ $rc -ne 0 ]; then tail -3 "$OUT/cfg_$name.err"; fi
  python3 -c "
import json
for l in open('$OUT/cfg_$name.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('   ', d['config'], d['stage'][:48], d['msps'], d.get('roofline',{}).get('frac'))
"
done
echo "exit 0"
