#!/bin/bash
# Round 6, first pass: the new parity cases (full-shape large-N grids, the streamed
# tail crossing), the recycled-buffer self-test, the ring tests, then the receiver bench.
set -o pipefail
TAG=${1:-r06a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export GSDR_PARITY_LOG=$OUT/parity_spread.jsonl
rm -f "$GSDR_PARITY_LOG"
echo "== recycled self-test" &&
GSDR_SELFTEST_ONLY=recycled timeout -k 10 180 ./gnss-sdr-new_amd/build/host_selftest tests/golden/GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat \
    > "$OUT/selftest_recycled.log" 2>&1; rc=$?; cat "$OUT/selftest_recycled.log"; [ $rc -eq 0 ] &&
echo "== tests" &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_acq_full_shapes.py tests/test_gpu_configs.py tests/test_gpu_stream.py \
    tests/test_host_mirror.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -15 "$OUT/pytest_gpu.log"; grep "parity acq" "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] &&
echo "== receiver" &&
for cfg in c3 c5; do for s in 1 0; do
    timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench $cfg 2 $s > "$OUT/receiver_${cfg}_s$s.json" \
        2> "$OUT/receiver_${cfg}_s$s.err" && cat "$OUT/receiver_${cfg}_s$s.json" || exit 1
done; done
rc=$?
echo "exit $rc"
exit $rc
