#!/bin/bash
# r04d: A/B of compile-time switches of the split / register four-step correlates
# (GSDR_SPLIT_TWF: the split's input factor as compile-time roots + one table read
# per column; GSDR_TW_TREE: baby-step / giant-step twiddle powers), each a library
# built with `make OUT=../build_ab/<name> EXTRA=-D...` and selected by GSDR_LIB:
# parity of the large-N paths per library, then the C3/C4/C5 acquisition lines and
# the C2 bench (20/5, no CPU baseline) per library.
#   gpurun --timeout 1200 -- bash profiles/gpu_r04d.sh TAG lib1 lib2 ...
set -o pipefail
TAG=${1:-r04d}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for LIB in "$@"; do
  name=$(basename $(dirname $LIB))
  echo "== parity $name"
  GSDR_LIB=$LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_acq_signals.py::test_large_fft_four_step \
      tests/test_gpu_acq_dwells.py::test_bit_transition_c4_four_step "tests/test_gpu_acq.py::test_packed_variants_match_oracle" \
      tests/test_gpu_acq.py::test_c2_synthetic_32prn -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
      > "$OUT/pytest_$name.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest_$name.log"; [ $rc -eq 0 ] || exit $rc
done
for LIB in "$@"; do
  name=$(basename $(dirname $LIB))
  echo "== configs $name"
  GSDR_LIB=$LIB GSDR_ACQ_SPLIT=2 GSDR_ACQ_SPLIT_ID=13 timeout -k 10 300 python -u profiles/configs_bench.py \
      --only C3,C4,C5 --acq-only --reps 6 > "$OUT/cfg_$name.jsonl" 2> "$OUT/cfg_$name.err" || exit 1
  python3 -c "
import json,sys
for l in open('$OUT/cfg_$name.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('   ', d['config'], d['stage'][:50], d['msps'], d.get('roofline',{}).get('frac'))
"
  echo "== c2 $name"
  GSDR_LIB=$LIB timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c2_$name.json" \
      2> "$OUT/c2_$name.err" || exit 1
  python3 -c "
import json
d=json.loads(open('$OUT/c2_$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('    c2', d['value'], 'corr us', r['avg_launch_us'], 'busy', r['busy_us_per_step'], 'frac', r['frac'])
"
done
