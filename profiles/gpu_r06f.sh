#!/bin/bash
# Round 6: the configuration tests and host self-tests on HEAD, the receiver bench
# (landed-items consumption with the cached landed index), then the QPW A/B.
set -o pipefail
TAG=${1:-r06f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== tests" &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_host_mirror.py tests/test_gpu_stream.py -m gpu -x -v \
    --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1; rc=$?; tail -4 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== receiver" &&
for cfg in c3 c5; do for s in 1 0; do
    timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench $cfg 2 $s > "$OUT/receiver_${cfg}_s$s.json" \
        2> "$OUT/receiver_${cfg}_s$s.err" || exit 1
    python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[1], r['msps'], r['real_time_factor'], r['host_seconds'])" "$OUT/receiver_${cfg}_s$s.json"
done; done
bash profiles/gpu_r06e.sh "$TAG/qpw"
