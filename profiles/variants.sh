#!/bin/bash
# Stage-isolation / scheduling variants of the bench (diagnostics, not the metric).
#   gpurun -- bash profiles/variants.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-var}
mkdir -p "$OUT"
for v in "" "--cu-partition" "--only acq" "--only trk"; do
    name=$(echo "default$v" | tr -d ' -')
    timeout -k 10 120 python bench.py --no-cpu-baseline $v > "$OUT/$name.json" 2> "$OUT/$name.err" || exit $?
    echo "$name: $(python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'], d.get('stages_us_per_launch'))")"
done
