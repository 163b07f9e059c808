set -o pipefail
mkdir -p gpurun_out/chains
timeout -k 10 400 python -u -m pytest tests/test_gpu_acq_two_step.py tests/test_gpu_acq_wipe.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/chains/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/chains/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/chains/pytest.log | head; exit $rc; }
for c in 2 4 1 2 4; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --acq-chains $c > gpurun_out/chains/c$c.json 2>/dev/null || exit $?
  python3 -c "
import json
d=json.loads(open('gpurun_out/chains/c$c.json').read().strip().splitlines()[-1]); r=d['roofline']
print('chains $c', d['value'], r['avg_launch_us'], r['busy_us_per_step'], d['components']['acq_only_msps'])
"
done
