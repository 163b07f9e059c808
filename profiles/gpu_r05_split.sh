#!/bin/bash
# Round 5: padded row layouts of the 25000-point split plans (ids 7 / 8) against the
# defaults (ids 1 / 4): parity first, then interleaved C5 acquisition lines.
#   gpurun -- bash profiles/gpu_r05_split.sh TAG
set -o pipefail
TAG=${1:-r05s}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_acq_signals.py -k "id7 or id8 or split" > "$OUT/pytest.txt" 2>&1 || { tail -20 "$OUT/pytest.txt"; exit 1; }
tail -2 "$OUT/pytest.txt"
ONLY=C5 bash profiles/gpu_cfg_ab.sh $TAG "base|GSDR_ACQ_SPLIT=1" "p7|GSDR_ACQ_SPLIT_ID=7" "p8|GSDR_ACQ_SPLIT_ID=8" \
    "base2|GSDR_ACQ_SPLIT=1" "p7b|GSDR_ACQ_SPLIT_ID=7" "p8b|GSDR_ACQ_SPLIT_ID=8"
