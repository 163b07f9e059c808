# sub-batch pipeline A/B: acquisition parity tests, then the C2 bench under the
# driver's flags with the pipeline (default, 1 handle) and without (GSDR_ACQ_PIPE=1)
set -o pipefail
OUT=gpurun_out/${1:-r03h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_acq.py tests/test_gpu_acq_dwells.py tests/test_gpu_acq_signals.py \
    tests/test_gpu_stream.py tests/test_gpu_acq_two_step.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_acq.log 2>&1
rc=$?; tail -2 $OUT/pytest_acq.log; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  timeout -k 10 200 "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || return 1
  python -c "import json;d=json.load(open('$OUT/bench_$tag.json'));r=d['roofline'];print('$tag', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'], r.get('busy_us_per_step'), r.get('launch_overlap'), d.get('components',{}).get('acq_only_msps'))"
}
for i in 1 2; do
run pipe4_$i python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline &&
run pipe1_$i env GSDR_ACQ_PIPE=1 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --acq-chains 2 &&
run pipe2_$i env GSDR_ACQ_PIPE=2 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
run pipe4_b128 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --blocks 128
