#!/bin/bash
# Round 6: the C2 / C5 lines with the clock warm-up (--min-warmup-ms 250, the default) under
# the driver's flags, twice, the same command under rocprofv3, and the multi-rank GPU test.
set -o pipefail
TAG=${1:-r06w}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 0 1; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/bench_$i.json') if l.startswith('{')][0])
print('c2', d['value'], d['ms_per_step'], 'corr us', d['roofline']['avg_launch_us'], 'frac', d['roofline']['frac'], d['prewarm'], d['check']['channels_within_25hz'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench_prof.json" 2> "$OUT/prof.err" || exit 1
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || exit 1
python3 -c "
import json
d=json.loads([l for l in open('$OUT/bench_c5.json') if l.startswith('{')][0])
print('c5', d['value'], d['real_time_factor'], d['prewarm'])"
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_multirank.log" 2>&1; rc=$?; tail -1 "$OUT/pytest_multirank.log"; exit $rc
