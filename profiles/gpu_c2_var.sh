#!/bin/bash
# C2 correlate variant A/B: the packed-variant parity tests, then the C2 bench (20/5)
# alternating GSDR_ACQ_CORR_VARIANT over the given ids, twice.
set -o pipefail
TAG=${1:-c2var}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_acq.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1; rc=$?
tail -2 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" "$OUT/pytest.log" | head; exit $rc; fi
for rep in 1 2; do
  for V in "$@"; do
    GSDR_ACQ_CORR_VARIANT=$V timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        > "$OUT/c2_v${V}_$rep.json" 2> "$OUT/c2_v${V}_$rep.err" || exit $?
    python3 -c "
import json
d=json.loads(open('$OUT/c2_v${V}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('v$V rep $rep', d['value'], 'corr', r['avg_launch_us'], 'busy', r['busy_us_per_step'], 'frac', r['frac'], 'acq_only', d['components']['acq_only_msps'])
"
  done
done
