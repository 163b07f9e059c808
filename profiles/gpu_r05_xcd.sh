#!/bin/bash
# Round 5: tracking pools with each handle's channels on one XCD (GSDR_TRK_XCD=1) against
# the default placement: tracking parity with the knob, then interleaved C3 / C5 tracking
# lines with per-phase timing.
#   gpurun -- bash profiles/gpu_r05_xcd.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r05x}
mkdir -p "$OUT"
GSDR_TRK_XCD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_trk.py tests/test_gpu_stream.py > "$OUT/pytest_xcd.txt" 2>&1 || { tail -20 "$OUT/pytest_xcd.txt"; exit 1; }
tail -1 "$OUT/pytest_xcd.txt"
for spec in "base|" "xcd|GSDR_TRK_XCD=1" "base2|" "xcd2|GSDR_TRK_XCD=1"; do
  IFS='|' read -r name ENVS <<< "$spec"
  env $ENVS GSDR_TRK_TIMING=2 timeout -k 10 200 python profiles/configs_bench.py --only C3,C5 --reps 3 \
      > "$OUT/cfg_$name.jsonl" 2> "$OUT/cfg_$name.err" || exit 1
  env $ENVS timeout -k 10 200 python profiles/configs_bench.py --only C3,C5 --reps 3 \
      > "$OUT/cfgnt_$name.jsonl" 2> "$OUT/cfgnt_$name.err" || exit 1
  echo "== $name"; grep "gsdr_trk timing" "$OUT/cfg_$name.err"; grep tracking "$OUT/cfgnt_$name.jsonl" | cut -c1-200
done
