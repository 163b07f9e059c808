#!/bin/bash
# r04e: round-4 checkpoint on HEAD's tree:
#  1. A/B of the twiddle switches (libraries built with EXTRA=-D..., GSDR_LIB):
#     C3/C4/C5 acquisition lines and the C2 bench (20/5) per library;
#  2. the C5 bench line (continuous tracking stream) and the drop-in receiver path
#     at configuration scale (host/tests/receiver_bench c3 / c5);
#  3. pytest -m gpu (the round's new parity checks: AVX / generic / fp64 per tap, C4 /
#     C5 at 45 dB-Hz, async ring windows, host self-test with blocking=false and the
#     acquisition dump).
# A stage that times out or crashes ends the script (no further GPU work).
#   gpurun --timeout 1200 -- bash profiles/gpu_r04e.sh TAG "name|lib|ENV=.. ENV=.." ...
set -o pipefail
TAG=${1:-r04e}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; }
for SPEC in "$@"; do
  IFS='|' read -r name LIB ENVS <<< "$SPEC"
  echo "== configs $name ($LIB $ENVS)"
  env $ENVS GSDR_LIB=$LIB timeout -k 10 240 python -u profiles/configs_bench.py --only C3,C4,C5 --acq-only --reps 6 \
      > "$OUT/cfg_$name.jsonl" 2> "$OUT/cfg_$name.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  python3 -c "
import json
for l in open('$OUT/cfg_$name.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('   ', d['config'], d['stage'][:48], d['msps'], d.get('roofline',{}).get('frac'))
"
  echo "== c2 $name"
  env $ENVS GSDR_LIB=$LIB timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c2_$name.json" \
      2> "$OUT/c2_$name.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  python3 -c "
import json
d=json.loads(open('$OUT/c2_$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('    c2', d['value'], 'corr us', r['avg_launch_us'], 'busy', r['busy_us_per_step'], 'frac', r['frac'], r.get('busy_source'))
"
done
echo "== c2 variant 71 (atomic row maxima), main library"
GSDR_ACQ_CORR_VARIANT=71 timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/c2_v71.json" 2> "$OUT/c2_v71.err"; rc=$?
if fatal $rc; then echo "fatal $rc"; exit $rc; fi
python3 -c "
import json
d=json.loads(open('$OUT/c2_v71.json').read().strip().splitlines()[-1]); r=d['roofline']
print('    c2 v71', d['value'], 'corr us', r['avg_launch_us'], 'busy', r['busy_us_per_step'], 'frac', r['frac'])
"
echo "== c5 bench (stream)"
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 5 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"; rc=$?
if fatal $rc; then echo "fatal $rc"; exit $rc; fi
tail -c 1500 "$OUT/bench_c5.json"
for c in c3 c5; do
  echo "== receiver_bench $c"
  timeout -k 10 240 ./gnss-sdr-new_amd/build/receiver_bench $c 0.4 > "$OUT/receiver_$c.json" 2> "$OUT/receiver_$c.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  cat "$OUT/receiver_$c.json"; tail -3 "$OUT/receiver_$c.err"
done
echo "== pytest -m gpu"
GSDR_PARITY_LOG=$OUT/parity_spread.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.txt" 2>&1; rc=$?
tail -15 "$OUT/pytest_gpu.txt"
exit $rc
