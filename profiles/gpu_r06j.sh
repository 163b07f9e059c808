#!/bin/bash
# Round 6: C2 bench with the two acquisition chains staggered (--acq-stagger S moves S blocks
# between the chains on alternate steps) against the default equal chains, alternating.
set -o pipefail
TAG=${1:-r06j}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for rep in 1 2; do for FL in "" "--acq-stagger 8" "--acq-stagger 4" "--acq-sizes 40,24"; do
  echo "== [$i] bench $FL"
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 $FL > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" \
      || { tail -5 "$OUT/bench_$i.err"; exit 1; }
  python3 -c "
import json,sys
for l in open('$OUT/bench_$i.json'):
    if l.startswith('{'):
        d=json.loads(l); print('$FL |', d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_us_per_launch'], d['components']['acq_only_msps'])"
  i=$((i + 1))
done; done
# 25000 plan A/B (GSDR_ACQ_25K_PLAN: 0 default 5-row rounds, 1 10-row rounds, 2 1024 lanes):
# parity under each alternative, then the C5 acquisition lines alternating
for PL in 1 2; do
  echo "== parity 25K plan $PL"
  GSDR_ACQ_25K_PLAN=$PL timeout -k 10 400 python -u -m pytest tests/test_gpu_acq_full_shapes.py tests/test_gpu_acq_signals.py \
      -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_25k_$PL.log" 2>&1 \
      || { tail -20 "$OUT/pytest_25k_$PL.log"; exit 1; }
  tail -1 "$OUT/pytest_25k_$PL.log"
done
bash profiles/ab_sweep.sh "$TAG/c5" "python -u profiles/configs_bench.py --only C5 --acq-only --reps 5" \
    "GSDR_ACQ_25K_PLAN=0" "GSDR_ACQ_25K_PLAN=1" "GSDR_ACQ_25K_PLAN=2" "GSDR_ACQ_25K_PLAN=0" "GSDR_ACQ_25K_PLAN=1" "GSDR_ACQ_25K_PLAN=2"
