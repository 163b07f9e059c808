set -o pipefail
OUT=gpurun_out/r03a
mkdir -p $OUT
export TMPDIR=/tmp
export GSDR_PARITY_LOG=$OUT/parity_spread.jsonl
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
echo "pytest rc $rc"
exit $rc
