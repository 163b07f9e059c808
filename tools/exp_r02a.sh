#!/bin/bash
# r02a: host self-test (new adapters, dwells, hand-off) + correlate-variant sweep.
set -o pipefail
OUT=gpurun_out/r02a
mkdir -p $OUT
export TMPDIR=/tmp
echo "== host_selftest"
timeout -k 10 180 ./gnss-sdr-new_amd/build/host_selftest tests/golden/GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat \
    tests/golden/Galileo_E1_ID_1_Fs_4Msps_8ms.dat > $OUT/host_selftest.log 2>&1
rc=$?
cat $OUT/host_selftest.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ] && exit $rc
for v in ${VARIANTS:-30 31 32 36 38 39}; do
  echo "== variant $v"
  GSDR_ACQ_CORR_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --only acq --steps 30 --warmup 10 \
      > $OUT/v$v.json 2>$OUT/v$v.err || { tail -5 $OUT/v$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/v$v.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'),d['check'])"
done
echo "== gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -15 $OUT/pytest_gpu.log
