#!/bin/bash
# r02d: ring tests + host self-test + the PMC passes (acq / trk / C3 separately).
set -o pipefail
OUT=gpurun_out/r02d
mkdir -p $OUT
export TMPDIR=/tmp
echo "== ring + host tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_host_mirror.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -25 $OUT/pytest.log
if [ $rc -ge 124 ]; then exit $rc; fi
echo "== pmc"
bash profiles/pmc_round2.sh r02d/pmc > $OUT/pmc_round.log 2>&1; tail -3 $OUT/pmc_round.log
