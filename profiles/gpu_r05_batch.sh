#!/bin/bash
# Round 5: receiver benches (tracking only) at pool batches 8 / 16 / 32, interleaved.
#   gpurun -- bash profiles/gpu_r05_batch.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r05bt}
mkdir -p "$OUT"
for rep in a b; do for cfg in c3 c5; do for b in 8 16 32; do
  timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench $cfg 2 0 1 $b > "$OUT/receiver_${cfg}_b${b}_$rep.json" \
      2> "$OUT/receiver_${cfg}_b${b}_$rep.err" || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/receiver_${cfg}_b${b}_$rep.json')); print('$cfg', $b, '$rep', d['msps'], d['host_seconds'], min(v['min_outputs_per_channel'] for v in d['signals'].values()))"
done; done; done
