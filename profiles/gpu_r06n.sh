#!/bin/bash
# Round 6: the receiver with the source running ahead of the blocks (lookahead 0 / 1 / 2
# chunks), C3 and C5, with and without the search.
set -o pipefail
TAG=${1:-r06n}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for la in 0 1 2; do for cfg in c3 c5; do for s in 0 1; do
    timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench $cfg 2 $s 1 0 $la > "$OUT/receiver_${cfg}_s${s}_la$la.json" \
        2> "$OUT/receiver_${cfg}_s${s}_la$la.err" || exit 1
    python3 -c "
import json; d=json.load(open('$OUT/receiver_${cfg}_s${s}_la$la.json'))
print('$cfg s$s la$la', d['msps'], d['real_time_factor'], {k: (v['channels_within_25hz'], v['channels'], v['min_outputs_per_channel']) for k, v in d['signals'].items()})"
done; done; done
