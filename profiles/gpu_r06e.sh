#!/bin/bash
# Round 6: 100000 = 4 x 25000 with two sub-transforms per 1024-lane workgroup sharing
# their products (GSDR_ACQ_QPW=2) against one per 512-lane workgroup (1): parity of
# the large-N plans under QPW 2, then the C5 acquisition lines alternating.
set -o pipefail
TAG=${1:-r06e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export GSDR_PARITY_LOG=$OUT/parity_spread.jsonl
L=gnss-sdr-new_amd/build_ab/qpw/libgsdr.so
echo "== parity (QPW 2)" &&
GSDR_LIB=$L GSDR_ACQ_QPW=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_acq_signals.py tests/test_gpu_acq_full_shapes.py \
    tests/test_gpu_acq_dwells.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.log" 2>&1; rc=$?; tail -4 "$OUT/pytest.log"; grep "parity acq" "$OUT/pytest.log"; [ $rc -eq 0 ] &&
bash profiles/ab_sweep.sh "$TAG/c5" "python -u profiles/configs_bench.py --only C5 --acq-only --reps 5" \
    "GSDR_LIB=$L GSDR_ACQ_QPW=1" "GSDR_LIB=$L GSDR_ACQ_QPW=2" "GSDR_LIB=$L GSDR_ACQ_QPW=1" "GSDR_LIB=$L GSDR_ACQ_QPW=2"
