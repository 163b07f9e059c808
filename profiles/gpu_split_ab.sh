#!/bin/bash
# r03 A/B: parity of every split of the large FFT sizes (incl. the forced
# 2 x 16000 / 4 x 16000 splits), of the packed N = 4000 variants (incl. the
# prime-factor 32 x 125 variant 80), the tracking dump fields (replay + host
# self-test); then the C2 bench under variants 70 / 80 and the C4/C5 acquisition
# lines under each split setting.
#   gpurun --timeout 1100 -- bash profiles/gpu_split_ab.sh TAG
set -o pipefail
TAG=${1:-r03q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== parity" &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_acq.py tests/test_gpu_acq_signals.py tests/test_gpu_acq_dwells.py \
    tests/test_gpu_trk.py tests/test_host_mirror.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; grep -E "tracking dump" "$OUT/pytest.log" | head -3; [ $rc -eq 0 ] || exit $rc
bash profiles/ab_sweep.sh "$TAG/c2" "python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline" \
    "GSDR_ACQ_CORR_VARIANT=70" "GSDR_ACQ_CORR_VARIANT=80" "GSDR_ACQ_CORR_VARIANT=70" "GSDR_ACQ_CORR_VARIANT=80" || exit 1
bash profiles/ab_sweep.sh "$TAG/big" "python -u profiles/configs_bench.py --only C4,C5 --reps 5" \
    "GSDR_ACQ_SPLIT=1" "GSDR_ACQ_SPLIT=2" "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=5" "GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=6"
