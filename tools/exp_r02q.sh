#!/bin/bash
# r02q: packed four-step (FourStepPkPlan, variants 24-27): acquisition parity at the
# four-step sizes (plain, dwells, bit transition, two-step, config tests), then C4
# acquisition timing with the packed and the generic four-step.
set -o pipefail
OUT=gpurun_out/r02q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_acq_signals.py tests/test_gpu_acq_dwells.py tests/test_gpu_acq_two_step.py tests/test_gpu_acq.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_acq.log 2>&1
rc=$?; tail -3 $OUT/pytest_acq.log; [ $rc -ne 0 ] && exit $rc
for g in 0 1; do
  echo "== C4 generic=$g"
  GSDR_ACQ_FOUR_GENERIC=$g timeout -k 10 300 python profiles/configs_bench.py --only C4 --reps 6 > $OUT/c4_g$g.jsonl 2> $OUT/c4_g$g.err || { tail -5 $OUT/c4_g$g.err; exit 1; }
  grep acquisition $OUT/c4_g$g.jsonl
done
echo done
