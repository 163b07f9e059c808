#!/bin/bash
# Round 5: kernel trace of the receiver bench (tracking only, C3 and C5): GPU time per
# advance launch against the host's wall time.
#   gpurun -- bash profiles/gpu_r05_recvprof.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r05rp}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv -- \
      ./gnss-sdr-new_amd/build/receiver_bench $cfg 2 0 > "$OUT/receiver_${cfg}.json" 2> "$OUT/receiver_${cfg}.err" || exit 1
  find "$OUT/prof_$cfg" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$cfg.csv" \;
  find "$OUT/prof_$cfg" -name "*memory_copy_stats.csv" -exec cp {} "$OUT/memcpy_stats_$cfg.csv" \; || true
  echo "== $cfg"; head -c 300 "$OUT/receiver_${cfg}.json"; echo; cut -d, -f1-8 "$OUT/kernel_stats_$cfg.csv" | cut -c1-220 | head -8
  cat "$OUT/memcpy_stats_$cfg.csv" 2>/dev/null | head -5
done
