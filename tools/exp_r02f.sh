#!/bin/bash
# r02f: host self-test (receiver on the device ring), config-rate tracking parity, full GPU suite.
set -o pipefail
OUT=gpurun_out/r02f
mkdir -p $OUT
export TMPDIR=/tmp
echo "== host_selftest"
timeout -k 10 120 ./gnss-sdr-new_amd/build/host_selftest tests/golden/GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat tests/golden/Galileo_E1_ID_1_Fs_4Msps_8ms.dat > $OUT/host_selftest.log 2>&1
rc=$?
grep -E "FAIL|ring|hand-off" $OUT/host_selftest.log; tail -2 $OUT/host_selftest.log
if [ $rc -ge 124 ]; then exit $rc; fi
echo "== config parity"
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_configs.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $OUT/pytest_configs.log | head -40; tail -3 $OUT/pytest_configs.log
if [ $rc -ge 124 ]; then exit $rc; fi
echo "== gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_configs.py > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
exit $rc
