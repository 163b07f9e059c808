#!/bin/bash
# Round 5: kernel + HIP runtime + copy trace of the C3 receiver bench (tracking only).
#   gpurun -- bash profiles/gpu_r05_recvtrace.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r05rt}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d "$OUT/prof" -o run --output-format csv -- \
    ./gnss-sdr-new_amd/build/receiver_bench c3 2 0 > "$OUT/receiver_c3.json" 2> "$OUT/receiver_c3.err"
rc=$?
ls -R "$OUT/prof" | head -20
exit $rc
