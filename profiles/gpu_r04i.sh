#!/bin/bash
# r04i: the split argmax pass (acq_correlate_split_kernel<ARG> + acq_argmax_split_finish_kernel):
# the large-N acquisition parity tests, then configs A/B (GSDR_ACQ_SPLIT_ARG=1 / 0).
set -o pipefail
TAG=${1:-r04i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; }
echo "== acq tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_acq_signals.py tests/test_gpu_acq_dwells.py tests/test_gpu_acq_wipe.py \
    tests/test_gpu_acq_two_step.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_acq.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_acq.log"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" "$OUT/pytest_acq.log" | head -20; exit $rc; fi
for SPEC in "arg|GSDR_ACQ_SPLIT_ARG=1" "old|GSDR_ACQ_SPLIT_ARG=0"; do
  IFS='|' read -r name ENVS <<< "$SPEC"
  echo "== configs $name"
  env $ENVS timeout -k 10 240 python -u profiles/configs_bench.py --only C4,C5 --acq-only --reps 6 \
      > "$OUT/cfg_$name.jsonl" 2> "$OUT/cfg_$name.err"; rc=$?
  if fatal $rc; then echo "fatal $rc"; exit $rc; fi
  python3 -c "
import json
for l in open('$OUT/cfg_$name.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('   ', d['config'], d['stage'][:48], d['msps'], d.get('roofline',{}).get('frac'))
"
done
echo "exit 0"
