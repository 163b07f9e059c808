#!/bin/bash
# r02c: GPU tests, the default bench line (with the C++ CPU baseline), the
# rocprofv3 kernel-trace summary of the same bench command, and the PMC passes.
set -o pipefail
OUT=gpurun_out/r02c
mkdir -p $OUT
export TMPDIR=/tmp
echo "== gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -4 $OUT/pytest_gpu.log
if [ $rc -ge 124 ]; then exit $rc; fi
echo "== smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; cat $OUT/smoke.log
echo "== bench"
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json || { tail -20 $OUT/bench.err; exit 1; }
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 20 > $OUT/bench_prof.json 2> $OUT/prof.err &&
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \; && cat $OUT/kernel_stats.csv | cut -c1-200 || exit 1
echo "== pmc"
bash profiles/pmc_round2.sh r02c/pmc > $OUT/pmc_round.log 2>&1; tail -3 $OUT/pmc_round.log
