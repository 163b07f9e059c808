# r03 split register four-step: acquisition parity tests, then the config lines
# with the split correlate (default) and the packed four-step (GSDR_ACQ_SPLIT=0)
set -o pipefail
OUT=gpurun_out/${1:-r03b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_acq_signals.py tests/test_gpu_acq_dwells.py tests/test_gpu_acq.py \
    tests/test_gpu_acq_two_step.py tests/test_gpu_stream.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_acq.log 2>&1
rc=$?; tail -3 $OUT/pytest_acq.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u profiles/configs_bench.py --only C3,C4,C5 --reps 5 > $OUT/configs_split.jsonl 2> $OUT/configs_split.err &&
GSDR_ACQ_SPLIT=0 timeout -k 10 300 python -u profiles/configs_bench.py --only C4,C5 --reps 5 > $OUT/configs_nosplit.jsonl 2> $OUT/configs_nosplit.err
rc=$?; grep acq $OUT/configs_split.jsonl $OUT/configs_nosplit.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
rc=$?; cat $OUT/bench_c5.json; tail -3 $OUT/bench_c5.err; exit $rc
