#!/bin/bash
# r02g: tracking-call breakdown (GSDR_TRK_TIMING=2: prep / correlate / update / window, wall clock ticks
# at 100 MHz) at C3 and C5, plus the C3 open-loop parity re-run.
set -o pipefail
OUT=gpurun_out/r02g
mkdir -p $OUT
export TMPDIR=/tmp
echo "== timing"
GSDR_TRK_TIMING=2 timeout -k 10 300 python profiles/configs_bench.py --only C3,C5 --reps 3 > $OUT/configs.jsonl 2> $OUT/timing.err
rc=$?
cat $OUT/configs.jsonl; grep -v "^$" $OUT/timing.err | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== c3 parity"
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 200 --timeout-method thread -k c3 > $OUT/pytest_c3.log 2>&1
rc=$?
tail -3 $OUT/pytest_c3.log
exit $rc
