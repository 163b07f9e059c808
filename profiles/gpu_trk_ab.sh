#!/bin/bash
# Tracking correlate A/B: tracking parity tests (open-loop taps, replay, configs, stream),
# then per-phase timing at C2 / C3 / C5 (gpu_trk_timing.sh notests) and the config lines.
#   gpurun -- bash profiles/gpu_trk_ab.sh TAG
set -o pipefail
TAG=${1:-r03v}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_trk.py tests/test_gpu_configs.py tests/test_gpu_stream.py tests/test_gpu_corr.py > "$OUT/pytest_trk.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_trk.log"; [ $rc -eq 0 ] || exit $rc
bash profiles/gpu_trk_timing.sh "$TAG" notests
