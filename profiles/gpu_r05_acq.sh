#!/bin/bash
# Round 5: acquisition parity suite after pruning the split alternatives, then the
# C3 / C4 / C5 acquisition lines.
#   gpurun -- bash profiles/gpu_r05_acq.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r05acq}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_acq_signals.py tests/test_gpu_acq_dwells.py tests/test_gpu_acq.py tests/test_gpu_acq_wipe.py \
    > "$OUT/pytest.txt" 2>&1 &&
timeout -k 10 300 python -u profiles/configs_bench.py --only C3,C4,C5 --acq-only --reps 6 > "$OUT/cfg.jsonl" 2> "$OUT/cfg.err"
rc=$?
tail -3 "$OUT/pytest.txt"
python3 -c "
import json
for l in open('$OUT/cfg.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['config'], d['stage'][:60], d['msps'], d.get('roofline',{}).get('frac'))
" 2>/dev/null
echo "exit $rc"
exit $rc
