#!/bin/bash
# Round 6: PMC passes of the C2 correlate on HEAD (the bench line's
# traffic source) and a kernel trace of the drop-in receiver with the search (item 4:
# is the GPU busy while the acquisition services run?).
set -o pipefail
TAG=${1:-r06c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash profiles/pmc_round2.sh "$TAG/pmc" > "$OUT/pmc_round.log" 2>&1; rc=$?; tail -3 "$OUT/pmc_round.log"; [ $rc -eq 0 ] &&
echo "== receiver c5 with search under the kernel trace" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/recv" -o run --output-format csv -- \
    ./gnss-sdr-new_amd/build/receiver_bench c5 2 1 > "$OUT/receiver_c5_s1_traced.json" 2> "$OUT/receiver_trace.err" &&
cat "$OUT/receiver_c5_s1_traced.json" &&
python3 profiles/kernel_union.py "$OUT/recv" > "$OUT/receiver_c5_s1_busy.json" && cat "$OUT/receiver_c5_s1_busy.json"
