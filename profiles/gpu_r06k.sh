#!/bin/bash
# Round 6: the lock test (CN0 estimate + lock detector) moved to wave 2 with wave 0 running
# the locked branch ahead of it. Tracking tests + host self-test on HEAD, then per-phase
# call timing and the tracking-only lines, HEAD vs the previous library, alternating.
set -o pipefail
TAG=${1:-r06k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B=gnss-sdr-new_amd/build_ab/base/libgsdr.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_trk.py tests/test_gpu_configs.py tests/test_gpu_stream.py tests/test_host_mirror.py > $OUT/pytest_trk.log 2>&1
rc=$?; tail -3 $OUT/pytest_trk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./gnss-sdr-new_amd/build/host_selftest tests/golden/GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat tests/golden/Galileo_E1_ID_1_Fs_4Msps_8ms.dat > $OUT/host_selftest.log 2>&1
rc=$?; tail -3 $OUT/host_selftest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for L in head0 head; do
  E=""; [ $L = head ] || E="GSDR_LIB=gnss-sdr-new_amd/build_ab/$L/libgsdr.so"
  echo "== $L timing"
  env $E GSDR_TRK_TIMING=2 timeout -k 10 200 python bench.py --only trk --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trk_${L}_$rep.json 2> $OUT/trk_${L}_$rep.err || exit 1
  grep "gsdr_trk timing" $OUT/trk_${L}_$rep.err | head -3
  env $E GSDR_TRK_TIMING=2 timeout -k 10 200 python profiles/configs_bench.py --only C5 --reps 3 > $OUT/cfg_${L}_$rep.jsonl 2> $OUT/cfg_${L}_$rep.err || exit 1
  grep "gsdr_trk timing" $OUT/cfg_${L}_$rep.err | head -6
  env $E timeout -k 10 200 python profiles/configs_bench.py --only C3,C5 --reps 3 > $OUT/cfgn_${L}_$rep.jsonl 2> $OUT/cfgn_${L}_$rep.err || exit 1
  grep -h tracking $OUT/cfgn_${L}_$rep.jsonl | cut -c1-260
done; done
