#!/bin/bash
# Round 6: short tracking calls (C2, 4000 samples) through the streamed path's LDS-DMA
# prefetch instead of the register-staged window (GSDR_TRK_WINDOW=0): parity under it, then
# per-phase timing and the tracking-only line alternating window 1 / 0.
set -o pipefail
TAG=${1:-r06r}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
GSDR_TRK_WINDOW=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
    tests/test_gpu_trk.py tests/test_gpu_configs.py tests/test_gpu_stream.py > $OUT/pytest_trk_w0.log 2>&1; rc=$?; tail -2 $OUT/pytest_trk_w0.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for W in 1 0; do
  echo "== window $W"
  GSDR_TRK_WINDOW=$W GSDR_TRK_TIMING=2 timeout -k 10 200 python bench.py --only trk --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trk_w${W}_$rep.json 2> $OUT/trk_w${W}_$rep.err || exit 1
  grep "gsdr_trk timing" $OUT/trk_w${W}_$rep.err | head -1 | cut -c1-400
  GSDR_TRK_WINDOW=$W timeout -k 10 200 python bench.py --only trk --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trkn_w${W}_$rep.json 2> $OUT/trkn_w${W}_$rep.err || exit 1
  python3 -c "
import json
for l in open('$OUT/trkn_w${W}_$rep.json'):
    if l.startswith('{'): d=json.loads(l); print('trk-only', d['value'], d['check']['channels_within_25hz'])"
done; done
