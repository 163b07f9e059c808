#!/bin/bash
# Round 6: the C2 tracking call's per-phase timing inside the full C2 step (acquisition grids
# running beside it, clocks ramped) against the tracking-only run.
set -o pipefail
TAG=${1:-r06y}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
GSDR_TRK_TIMING=2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/full.json" 2> "$OUT/full.err" || exit 1
grep "gsdr_trk timing" "$OUT/full.err" | head -2 | cut -c1-420
GSDR_TRK_TIMING=2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --only trk > "$OUT/trk.json" 2> "$OUT/trk.err" || exit 1
grep "gsdr_trk timing" "$OUT/trk.err" | head -2 | cut -c1-420
