set -o pipefail
# Tracking iteration on the GPU box: tracking parity tests, the host self-test,
# then per-phase call timing (GSDR_TRK_TIMING=2) at C2 (bench trk leg) and C3/C5.
# usage: bash profiles/gpu_trk_timing.sh TAG [notests]
OUT=gpurun_out/${1:-r03k}
mkdir -p $OUT
if [ "$2" != "notests" ]; then
    timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
        tests/test_gpu_trk.py tests/test_gpu_configs.py tests/test_gpu_stream.py > $OUT/pytest_trk.log 2>&1
    rc=$?; tail -3 $OUT/pytest_trk.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 ./gnss-sdr-new_amd/build/host_selftest tests/golden/GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat tests/golden/Galileo_E1_ID_1_Fs_4Msps_8ms.dat > $OUT/host_selftest.log 2>&1
rc=$?; tail -4 $OUT/host_selftest.log; [ $rc -eq 0 ] || exit $rc
GSDR_TRK_TIMING=2 timeout -k 10 200 python bench.py --only trk --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trk_only.json 2> $OUT/trk_only.err || exit 1
grep "gsdr_trk timing" $OUT/trk_only.err
timeout -k 10 200 python bench.py --only trk --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trk_only_notiming.json 2>&1 || exit 1
tail -c 400 $OUT/trk_only_notiming.json
GSDR_TRK_TIMING=2 timeout -k 10 200 python profiles/configs_bench.py --only C3,C5 --reps 3 > $OUT/cfg.jsonl 2> $OUT/cfg.err || exit 1
grep "gsdr_trk timing" $OUT/cfg.err; grep tracking $OUT/cfg.jsonl
timeout -k 10 200 python profiles/configs_bench.py --only C3,C5 --reps 3 > $OUT/cfg_notiming.jsonl 2> $OUT/cfg_notiming.err || exit 1
grep tracking $OUT/cfg_notiming.jsonl
