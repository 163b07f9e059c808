#!/bin/bash
# Round 5: the receiver benches only (host-time breakdown in the JSON lines).
#   gpurun -- bash profiles/gpu_r05_recv.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r05r}
mkdir -p "$OUT"
for cfg in c3 c5; do for s in 0 1; do
  timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench $cfg 2 $s > "$OUT/receiver_${cfg}_s$s.json" \
      2> "$OUT/receiver_${cfg}_s$s.err" || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/receiver_${cfg}_s$s.json')); print('$cfg', $s, d['msps'], d['seconds'], d['host_seconds'])"
done; done
