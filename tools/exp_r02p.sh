#!/bin/bash
# r02p: DPP wave max + buffer-descriptor row loads + clamped single-pass stage loads
# in the packed correlate kernel: acquisition parity, acquisition-only bench of the
# default variant and 31, then the full bench line.
set -o pipefail
OUT=gpurun_out/r02p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_acq.py tests/test_gpu_acq_dwells.py tests/test_gpu_acq_two_step.py tests/test_gpu_acq_signals.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_acq.log 2>&1
rc=$?; tail -3 $OUT/pytest_acq.log; [ $rc -ne 0 ] && exit $rc
for v in 70 31; do
  echo "== variant $v"
  GSDR_ACQ_CORR_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --only acq > $OUT/v$v.json 2> $OUT/v$v.err || { tail -5 $OUT/v$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/v$v.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'))"
done
echo "== bench"
timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'),d['check'])"
