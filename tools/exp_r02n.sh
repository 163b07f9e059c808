#!/bin/bash
# r02n: HEAD round (tests, smoke, bench, rocprof), then the correlate variants of the
# experimental build (build/exp/libgsdr.so): acquisition-only bench per variant and
# acquisition parity on the new max-only / per-stage-twiddle variants.
set -o pipefail
OUT=gpurun_out/r02n
mkdir -p $OUT
export TMPDIR=/tmp
bash profiles/gpu_round.sh r02m || exit 1
export GSDR_LIB=$PWD/gnss-sdr-new_amd/build/exp/libgsdr.so
for v in ${VARIANTS:-31 70 71 72 73 74}; do
  echo "== variant $v"
  GSDR_ACQ_CORR_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --only acq > $OUT/v$v.json 2> $OUT/v$v.err || { tail -5 $OUT/v$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/v$v.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'))"
done
for v in ${PVARIANTS:-72 74}; do
  echo "== parity variant $v"
  GSDR_ACQ_CORR_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_acq.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_v$v.log 2>&1
  rc=$?; tail -3 $OUT/pytest_v$v.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
