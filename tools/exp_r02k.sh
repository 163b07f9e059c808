#!/bin/bash
# r02k: tracking parity after the update rewrite (LDS-ordered CN0 sums), then timing
set -o pipefail
OUT=gpurun_out/${TAG:-r02k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_trk.py tests/test_gpu_stream.py tests/test_host_mirror.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_trk.log 2>&1
rc=$?
tail -3 $OUT/pytest_trk.log
[ $rc -ne 0 ] && exit $rc
GSDR_TRK_TIMING=2 timeout -k 10 300 python profiles/configs_bench.py --only ${ONLY:-C3,C4,C5} --reps 5 > $OUT/configs_timing.jsonl 2> $OUT/timing.err
rc=$?
grep "gsdr_trk timing" $OUT/timing.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python profiles/configs_bench.py --only ${ONLY:-C3,C4,C5} --reps 10 > $OUT/configs.jsonl 2> $OUT/configs.err
rc=$?
cat $OUT/configs.jsonl
exit $rc
