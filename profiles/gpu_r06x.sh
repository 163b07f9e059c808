#!/bin/bash
# Round 6: the per-configuration lines with the clock warm-up (--warm-ms 250, the default)
# against --warm-ms 0, on one box.
set -o pipefail
TAG=${1:-r06x}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u profiles/configs_bench.py --reps 5 --warm-ms 0 > "$OUT/configs_cold.jsonl" 2> "$OUT/configs_cold.err" || exit 1
timeout -k 10 400 python -u profiles/configs_bench.py --reps 5 > "$OUT/configs.jsonl" 2> "$OUT/configs.err" || exit 1
python3 - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
def rows(f):
    r = {}
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l); r[(d.get('config'), d.get('stage', '')[:60])] = (d.get('msps'), (d.get('roofline') or {}).get('frac'))
    return r
c, w = rows(out + '/configs_cold.jsonl'), rows(out + '/configs.jsonl')
for k in w:
    print(k[0], k[1], '| cold', c.get(k), '| warm', w[k])
PY
