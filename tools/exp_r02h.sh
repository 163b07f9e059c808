#!/bin/bash
# r02h: LDS-streamed tracking calls (vector_length > 4096): parity (tracking tests, config tests) then timing.
set -o pipefail
OUT=gpurun_out/${TAG:-r02h}
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tracking parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_trk.py tests/test_gpu_stream.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_trk.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $OUT/pytest_trk.log | head -60; tail -3 $OUT/pytest_trk.log
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== timing"
GSDR_TRK_TIMING=2 timeout -k 10 300 python profiles/configs_bench.py --only C3,C4,C5 --reps 5 > $OUT/configs.jsonl 2> $OUT/timing.err
rc=$?
cat $OUT/configs.jsonl; grep "gsdr_trk timing" $OUT/timing.err
[ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['stages_us_per_launch'],d['check'])"
exit $rc
