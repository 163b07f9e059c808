#!/bin/bash
# Round 6: the receiver with the tracking blocks' work() on T threads (GNU Radio runs every
# block on its own thread), T = 0 (one thread) / 2 / 4 / 8, C3 and C5, with and without search.
set -o pipefail
TAG=${1:-r06o}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for th in 0 2 4 8; do for cfg in c3 c5; do for s in 0 1; do
    f="$OUT/receiver_${cfg}_s${s}_t$th"
    timeout -k 10 120 ./gnss-sdr-new_amd/build/receiver_bench $cfg 2 $s 1 0 0 $th > "$f.json" 2> "$f.err" || { echo "rc=$? $f"; tail -5 "$f.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$f.json'))
print('$cfg s$s t$th', d['msps'], d['real_time_factor'], d['trk_work_calls'], {k: (v['channels_within_25hz'], v['channels'], v['min_outputs_per_channel'], v['outputs']) for k, v in d['signals'].items()})"
done; done; done
