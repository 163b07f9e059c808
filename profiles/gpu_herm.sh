#!/bin/bash
# Mirror-pair (Hermitian code) split correlate: parity tests, then the C3/C4/C5
# acquisition lines with GSDR_ACQ_HERM=1 (default) and =0, interleaved.
#   gpurun --timeout 900 -- bash profiles/gpu_herm.sh TAG
set -o pipefail
TAG=${1:-herm}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_acq_signals.py tests/test_gpu_acq_two_step.py tests/test_gpu_acq_wipe.py \
    > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
bash profiles/gpu_cfg_ab.sh $TAG "herm1|GSDR_ACQ_HERM=1" "herm0|GSDR_ACQ_HERM=0" "herm1b|GSDR_ACQ_HERM=1" "herm0b|GSDR_ACQ_HERM=0"
