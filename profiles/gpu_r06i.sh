#!/bin/bash
# Round 6: two acquisition launches in flight per service (gsdr_acq_submit_stream queue
# depth 2): stream / host-mirror tests, the receiver with search, then parity under
# GSDR_ACQ_PPW=2 and the C5 acquisition A/B (one vs two PRNs per 25000 workgroup).
set -o pipefail
TAG=${1:-r06i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== stream + host mirror tests" &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_host_mirror.py -m gpu -x -v --timeout 200 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest_stream.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_stream.log"; [ $rc -eq 0 ] &&
echo "== receiver" &&
for cfg in c3 c5; do for s in 1 0; do
    timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench $cfg 2 $s > "$OUT/receiver_${cfg}_s$s.json" \
        2> "$OUT/receiver_${cfg}_s$s.err" && cat "$OUT/receiver_${cfg}_s$s.json" || exit 1
done; done &&
echo "== parity (PPW 2)" &&
GSDR_PARITY_LOG=$OUT/parity_spread.jsonl GSDR_ACQ_PPW=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_acq_signals.py \
    tests/test_gpu_acq_full_shapes.py tests/test_gpu_acq_dwells.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_ppw2.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_ppw2.log"; [ $rc -eq 0 ] &&
bash profiles/ab_sweep.sh "$TAG/c5" "python -u profiles/configs_bench.py --only C5 --acq-only --reps 5" \
    "GSDR_ACQ_PPW=1" "GSDR_ACQ_PPW=2" "GSDR_ACQ_PPW=1" "GSDR_ACQ_PPW=2"
