#!/bin/bash
# r02e: config-rate tracking parity (C1-C5), correlator parity with E1 codes, and the
# per-config throughput lines (profiles/configs_bench.py).
set -o pipefail
OUT=gpurun_out/r02e
mkdir -p $OUT
export TMPDIR=/tmp
echo "== config parity"
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_corr.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $OUT/pytest.log | head -40; tail -3 $OUT/pytest.log
if [ $rc -ge 124 ]; then exit $rc; fi
echo "== configs"
timeout -k 10 400 python profiles/configs_bench.py > $OUT/configs.jsonl 2> $OUT/configs.err; cat $OUT/configs.jsonl; tail -3 $OUT/configs.err
