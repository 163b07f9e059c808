#!/bin/bash
# r02t: full GPU test suite on the packed four-step build, then C3/C4/C5 config lines
set -o pipefail
OUT=gpurun_out/r02t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python profiles/configs_bench.py --reps 10 > $OUT/configs.jsonl 2> $OUT/configs.err || { tail -5 $OUT/configs.err; exit 1; }
cat $OUT/configs.jsonl
