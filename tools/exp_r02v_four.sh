#!/bin/bash
# A/B of the four-step correlate variants on C4 (N = 64000: 25 default, 28 no prefetch,
# 29 two-column phase 1) and C5 (N = 25000: 27 default, 23 two-column phase 1).
set -o pipefail
O=gpurun_out/four; mkdir -p $O
for v in 25 28 29 25 29; do
  echo "variant $v" >> $O/c4.jsonl
  GSDR_ACQ_FOUR_VARIANT=$v timeout -k 10 200 python -u profiles/configs_bench.py --only C4 --reps 6 2>>$O/err.log | grep acquisition >> $O/c4.jsonl || exit 1
done
for v in 27 23 27 23; do
  echo "variant $v" >> $O/c5.jsonl
  GSDR_ACQ_FOUR_VARIANT=$v timeout -k 10 200 python -u profiles/configs_bench.py --only C5 --reps 6 2>>$O/err.log | grep "acquisition GPS" >> $O/c5.jsonl || exit 1
done
cat $O/c4.jsonl $O/c5.jsonl
