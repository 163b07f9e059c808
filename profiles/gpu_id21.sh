set -o pipefail
mkdir -p gpurun_out/id21
GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=21 timeout -k 10 300 python -u -m pytest tests/test_gpu_acq_signals.py -m gpu -x -q -k "100000 and id21" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/id21/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/id21/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/id21/pytest.log | head; exit $rc; }
for spec in "def|GSDR_ACQ_SPLIT=1" "id21|GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=21" "def2|GSDR_ACQ_SPLIT=1" "id21b|GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=21"; do
  IFS='|' read -r name ENVS <<< "$spec"
  env $ENVS timeout -k 10 240 python -u profiles/configs_bench.py --only C5 --acq-only --reps 6 > gpurun_out/id21/cfg_$name.jsonl 2> gpurun_out/id21/cfg_$name.err || exit $?
  python3 -c "
import json
for l in open('gpurun_out/id21/cfg_$name.jsonl'):
    if l.startswith('{') and '100000' in l:
        d=json.loads(l); print('$name', d['stage'][:40], d['msps'], d['roofline']['frac'])
"
done
