#!/bin/bash
# Round 6: where wave 2's lock test spends the C2 / C5 call (GSDR_TRK_TIMING=2 with the
# wave-2 probes), plus the tracking tests.
set -o pipefail
TAG=${1:-r06q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_trk.py tests/test_gpu_configs.py > $OUT/pytest_trk.log 2>&1; rc=$?; tail -2 $OUT/pytest_trk.log; [ $rc -eq 0 ] || exit $rc
GSDR_TRK_TIMING=2 timeout -k 10 200 python bench.py --only trk --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trk.json 2> $OUT/trk.err || exit 1
grep "gsdr_trk timing" $OUT/trk.err | head -3
GSDR_TRK_TIMING=2 timeout -k 10 200 python profiles/configs_bench.py --only C5 --reps 3 > $OUT/cfg.jsonl 2> $OUT/cfg.err || exit 1
grep "gsdr_trk timing" $OUT/cfg.err | head -4
