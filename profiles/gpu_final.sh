#!/bin/bash
# The driver's round-end checks on HEAD: every -m gpu test, smoke, the default bench line.
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export GSDR_PARITY_LOG=$OUT/parity_spread.jsonl
rm -f "$GSDR_PARITY_LOG"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && cat "$OUT/smoke.log" &&
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && cut -c1-200 "$OUT/bench.json"
