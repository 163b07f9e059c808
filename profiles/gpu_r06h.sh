#!/bin/bash
# Round 6: 25000 with two PRNs per 1024-lane workgroup sharing the X row's copies
# (GSDR_ACQ_PPW=2) against one PRN per 512-lane workgroup (1): parity under PPW 2, then
# the C5 acquisition lines alternating.
set -o pipefail
TAG=${1:-r06h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export GSDR_PARITY_LOG=$OUT/parity_spread.jsonl
L=gnss-sdr-new_amd/build_ab/ppw/libgsdr.so
echo "== parity (PPW 2)" &&
GSDR_LIB=$L GSDR_ACQ_PPW=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_acq_signals.py tests/test_gpu_acq_full_shapes.py \
    tests/test_gpu_acq_dwells.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.log" 2>&1; rc=$?; tail -4 "$OUT/pytest.log"; grep "parity acq" "$OUT/pytest.log"; [ $rc -eq 0 ] &&
bash profiles/ab_sweep.sh "$TAG/c5" "python -u profiles/configs_bench.py --only C5 --acq-only --reps 5" \
    "GSDR_LIB=$L GSDR_ACQ_PPW=1" "GSDR_LIB=$L GSDR_ACQ_PPW=2" "GSDR_LIB=$L GSDR_ACQ_PPW=1" "GSDR_LIB=$L GSDR_ACQ_PPW=2"
