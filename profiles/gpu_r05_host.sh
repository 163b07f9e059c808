#!/bin/bash
# Round 5: the drop-in receiver path after the Gnss_Synchro / batching changes, and
# the acquisition parity suite after the pruning of the measured losers.
#   gpurun -- bash profiles/gpu_r05_host.sh TAG [extra pytest files...]
set -o pipefail
OUT=gpurun_out/${1:-r05a}
shift
mkdir -p "$OUT/synchro"
GSDR_SELFTEST_ONLY=synchro GSDR_SELFTEST_DUMP_DIR="$OUT/synchro" timeout -k 10 120 \
    ./gnss-sdr-new_amd/build/host_selftest tests/golden/GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat > "$OUT/synchro.txt" 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_host_mirror.py tests/test_gpu_trk.py "$@" > "$OUT/pytest.txt" 2>&1 &&
timeout -k 10 200 ./gnss-sdr-new_amd/build/receiver_bench c3 2 1 > "$OUT/receiver_c3_s1.json" 2> "$OUT/receiver_c3_s1.err" &&
timeout -k 10 200 ./gnss-sdr-new_amd/build/receiver_bench c3 2 0 > "$OUT/receiver_c3_s0.json" 2> "$OUT/receiver_c3_s0.err" &&
timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench c5 2 1 > "$OUT/receiver_c5_s1.json" 2> "$OUT/receiver_c5_s1.err" &&
timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench c5 2 0 > "$OUT/receiver_c5_s0.json" 2> "$OUT/receiver_c5_s0.err" &&
timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench c5 2 0 0 > "$OUT/receiver_c5_s0_pageable.json" 2> "$OUT/receiver_c5_s0_pageable.err"
rc=$?
tail -5 "$OUT/pytest.txt"
cat "$OUT"/receiver_*.json
echo "exit $rc"
exit $rc
