set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
timeout -k 10 200 ./gnss-sdr-new_amd/build/host_selftest tests/golden/GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat tests/golden/Galileo_E1_ID_1_Fs_4Msps_8ms.dat > $OUT/host_selftest.log 2>&1
rc=$?; tail -4 $OUT/host_selftest.log; [ $rc -eq 0 ] || exit $rc
GSDR_TRK_TIMING=2 timeout -k 10 200 python bench.py --only trk --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trk_only.json 2> $OUT/trk_only.err || exit 1
grep "gsdr_trk timing" $OUT/trk_only.err
GSDR_TRK_TIMING=2 timeout -k 10 200 python profiles/configs_bench.py --only C3,C5 --reps 3 > $OUT/cfg.jsonl 2> $OUT/cfg.err || exit 1
grep "gsdr_trk timing" $OUT/cfg.err; grep tracking $OUT/cfg.jsonl
