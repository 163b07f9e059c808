#!/bin/bash
# Round 5: streamed tracking calls with 2 / 3 / default LDS chunk buffers
# (GSDR_TRK_STREAM_BUFS), C3 / C5 tracking lines with per-phase timing.
#   gpurun -- bash profiles/gpu_r05_bufs.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r05b}
mkdir -p "$OUT"
for spec in "b2|GSDR_TRK_STREAM_BUFS=2" "b3|GSDR_TRK_STREAM_BUFS=3" "b3c8|GSDR_TRK_STREAM_BUFS=3 GSDR_TRK_STREAM_CHUNK=8192" "def|"; do
  IFS='|' read -r name ENVS <<< "$spec"
  env $ENVS GSDR_TRK_TIMING=2 timeout -k 10 200 python profiles/configs_bench.py --only C3,C5 --reps 3 \
      > "$OUT/cfg_$name.jsonl" 2> "$OUT/cfg_$name.err" || exit 1
  env $ENVS timeout -k 10 200 python profiles/configs_bench.py --only C3,C5 --reps 3 \
      > "$OUT/cfgnt_$name.jsonl" 2> "$OUT/cfgnt_$name.err" || exit 1
  echo "== $name"; grep "gsdr_trk timing" "$OUT/cfg_$name.err" | cut -c1-230; grep tracking "$OUT/cfgnt_$name.jsonl" | cut -c1-170
done
