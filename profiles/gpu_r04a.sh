#!/bin/bash
# r04a: wave-local row transforms for the large-N correlates (acq_split.hip ids
# 11-20, C3 variant 94): parity of every new plan, then the C3/C4/C5 acquisition
# lines under each plan.
#   gpurun --timeout 1100 -- bash profiles/gpu_r04a.sh TAG
set -o pipefail
TAG=${1:-r04a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== parity" &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_acq_signals.py::test_large_fft_four_step \
    tests/test_gpu_acq_dwells.py::test_bit_transition_c4_four_step "tests/test_gpu_acq.py::test_packed_variants_match_oracle" \
    -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -5 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
bash profiles/ab_sweep.sh "$TAG/big" "python -u profiles/configs_bench.py --only C3,C4,C5 --acq-only --reps 6" \
    "GSDR_ACQ_SPLIT=2" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=11 GSDR_ACQ_CORR_VARIANT=94" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=12" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=13" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=14" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=15" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=16" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=17" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=18" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=19" \
    "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=20" \
    "GSDR_ACQ_SPLIT=1"
echo "== stream + host mirror" &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_host_mirror.py -x -v \
    --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_host.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_host.log"; exit $rc
