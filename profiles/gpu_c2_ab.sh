#!/bin/bash
# C2 correlate A/B: parity of the packed N = 4000 variants, then the bench line
# under each GSDR_ACQ_CORR_VARIANT given (alternating, driver flags).
#   gpurun --timeout 900 -- bash profiles/gpu_c2_ab.sh TAG 70 81 70 81
set -o pipefail
TAG=${1:-r03r}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== parity" &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_acq.py tests/test_gpu_acq_dwells.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
SETTINGS=()
for v in "$@"; do SETTINGS+=("GSDR_ACQ_CORR_VARIANT=$v"); done
bash profiles/ab_sweep.sh "$TAG" "python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline" "${SETTINGS[@]}"
