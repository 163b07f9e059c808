#!/bin/bash
# Correlate-kernel variant sweep + acquisition parity under a chosen variant.
set -o pipefail
OUT=gpurun_out/${1:-pk}
V=${2:-32}
mkdir -p "$OUT"
timeout -k 10 300 python3 profiles/sweep_corr.py ${3:-30,35,37} > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err" &&
cat "$OUT/sweep.jsonl" &&
GSDR_ACQ_CORR_VARIANT=$V timeout -k 10 300 python3 -u -m pytest tests/test_gpu_acq.py -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_acq.log" 2>&1; tail -3 "$OUT/pytest_acq.log"
