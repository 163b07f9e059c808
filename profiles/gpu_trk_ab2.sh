#!/bin/bash
# Tracking A/B per spec "name|lib": tracking parity tests, configs lines (tracking + acquisition),
# and the C2 bench components, with GSDR_LIB=lib.
set -o pipefail
TAG=${1:-trkab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; }
for SPEC in "$@"; do
  IFS='|' read -r name LIB <<< "$SPEC"
  echo "== $name tests ($LIB)"
  env ${LIB:+GSDR_LIB=$LIB} timeout -k 10 400 python -u -m pytest tests/test_gpu_trk.py tests/test_gpu_configs.py -m gpu -x -q \
      --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$name.log" 2>&1; rc=$?
  tail -2 "$OUT/pytest_$name.log"
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" "$OUT/pytest_$name.log" | head; exit $rc; fi
  echo "== $name configs"
  env ${LIB:+GSDR_LIB=$LIB} timeout -k 10 300 python -u profiles/configs_bench.py --only C3,C4,C5 --reps 5 > "$OUT/cfg_$name.jsonl" \
      2> "$OUT/cfg_$name.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  python3 -c "
import json
for l in open('$OUT/cfg_$name.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('   ', d['config'], d['stage'][:60], d['msps'], d.get('real_time_factor'))
"
  echo "== $name c2"
  env ${LIB:+GSDR_LIB=$LIB} timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c2_$name.json" \
      2> "$OUT/c2_$name.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  python3 -c "
import json
d=json.loads(open('$OUT/c2_$name.json').read().strip().splitlines()[-1])
print('    c2', d['value'], d['components'].get('trk_only_msps'), d['components'].get('acq_only_msps'), d['check'].get('channels_within_25hz'))
"
done
echo "exit 0"
