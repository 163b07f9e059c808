#!/bin/bash
# r02b: host self-test + GPU tests + default bench (variant 31 default).
set -o pipefail
OUT=gpurun_out/r02b
mkdir -p $OUT
export TMPDIR=/tmp
echo "== host_selftest"
timeout -k 10 180 ./gnss-sdr-new_amd/build/host_selftest tests/golden/GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat \
    tests/golden/Galileo_E1_ID_1_Fs_4Msps_8ms.dat > $OUT/host_selftest.log 2>&1
rc=$?
cat $OUT/host_selftest.log
if [ $rc -ge 124 ]; then exit $rc; fi
echo "== gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -15 $OUT/pytest_gpu.log
if [ $rc -ge 124 ]; then exit $rc; fi
echo "== bench"
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json
