#!/bin/bash
# Outer-DIF pre-pass (GSDR_ACQ_PRE=C: C PRNs per chunk, two buffers, the next chunk's pass on a
# second stream overlapping this chunk's grid pass): the large-FFT parity tests incl. the
# pre1 / pre64 variants, then the C4/C5 acquisition lines over the given specs.
#   gpurun --timeout 900 -- bash profiles/gpu_pre.sh TAG "name|ENV=.." ...
set -o pipefail
TAG=${1:-pre}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_acq_signals.py -k "large_fft" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
ONLY=C4,C5 bash profiles/gpu_cfg_ab.sh $TAG "$@"
