#!/bin/bash
# Round 6: the staged (LDS-DMA) phase 1 of the ROUT > 1 split correlates against the
# VGPR form: parity of every large-N plan with the staged build, then the C4 / C5
# acquisition lines under each build, interleaved.
set -o pipefail
TAG=${1:-r06b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export GSDR_PARITY_LOG=$OUT/parity_spread.jsonl
B=gnss-sdr-new_amd/build_ab
echo "== parity (staged build)" &&
GSDR_LIB=$B/dma4all/libgsdr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_acq_signals.py tests/test_gpu_acq_dwells.py \
    tests/test_gpu_acq_full_shapes.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.log" 2>&1; rc=$?; tail -4 "$OUT/pytest.log"; grep "parity acq" "$OUT/pytest.log"; [ $rc -eq 0 ] &&
bash profiles/ab_sweep.sh "$TAG/big" "python -u profiles/configs_bench.py --only C4,C5 --acq-only --reps 5" \
    "GSDR_LIB=$B/nodma/libgsdr.so" "GSDR_LIB=$B/dma4/libgsdr.so" "GSDR_LIB=$B/dma4all/libgsdr.so" \
    "GSDR_LIB=$B/dma6all/libgsdr.so" "GSDR_LIB=$B/nodma/libgsdr.so" "GSDR_LIB=$B/dma4all/libgsdr.so" &&
echo "== rocFFT A/B (the library path for the large-N grids)" &&
timeout -k 10 300 ./gnss-sdr-new_amd/build/rocfft_ab 5 > "$OUT/rocfft_ab.jsonl" 2> "$OUT/rocfft_ab.err"; rc=$?; cat "$OUT/rocfft_ab.jsonl"; tail -3 "$OUT/rocfft_ab.err"; exit $rc
