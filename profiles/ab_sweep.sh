#!/bin/bash
# A/B sweep on the GPU box (replaces round 2's one-off tools/exp_r02*.sh scripts):
# one command (bench.py or profiles/configs_bench.py) under each environment
# setting given, each run under its own time limit, the chain stopping at the
# first failure.  Results: gpurun_out/$TAG/ab_<i>.json (+ .err), summary lines.
#   gpurun -- bash profiles/ab_sweep.sh TAG "python bench.py --steps 20 --warmup 5" \
#       "GSDR_ACQ_SPLIT=0" "GSDR_ACQ_SPLIT=1"
#   gpurun -- bash profiles/ab_sweep.sh TAG "python profiles/configs_bench.py --only C5" "GSDR_ACQ_CORR_VARIANT=93"
set -o pipefail
TAG=$1; CMD=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for SETTING in "$@"; do
  echo "== [$i] $SETTING :: $CMD"
  timeout -k 10 300 env $SETTING $CMD > "$OUT/ab_$i.json" 2> "$OUT/ab_$i.err" || { tail -5 "$OUT/ab_$i.err"; exit 1; }
  PYTHONIOENCODING=utf-8 python3 - "$OUT/ab_$i.json" "$SETTING" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    r = d.get("roofline", {})
    print(sys.argv[2], "|", d.get("stage", d.get("metric", ""))[:60], "|", d.get("value", d.get("msps")),
          "| frac", r.get("frac"), "| launch us", r.get("avg_launch_us"))
PY
  i=$((i + 1))
done
