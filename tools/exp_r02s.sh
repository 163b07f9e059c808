#!/bin/bash
# r02s: packed four-step with / without the phase-2 prefetch (variants 25 / 28 at N = 64000)
set -o pipefail
OUT=gpurun_out/r02s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_acq_signals.py tests/test_gpu_acq_dwells.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_acq.log 2>&1
rc=$?; tail -3 $OUT/pytest_acq.log; [ $rc -ne 0 ] && exit $rc
for v in 25 28; do
  echo "== C4 four-step variant $v"
  GSDR_ACQ_FOUR_VARIANT=$v timeout -k 10 300 python profiles/configs_bench.py --only C4 --reps 6 > $OUT/c4_v$v.jsonl 2> $OUT/c4_v$v.err || { tail -5 $OUT/c4_v$v.err; exit 1; }
  grep acquisition $OUT/c4_v$v.jsonl
done
echo done
