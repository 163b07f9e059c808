#!/bin/bash
# tracking-call breakdown (GSDR_TRK_TIMING=2) at C3/C4/C5
set -o pipefail
OUT=gpurun_out/${TAG:-timing}
mkdir -p $OUT
export TMPDIR=/tmp
GSDR_TRK_TIMING=2 timeout -k 10 300 python profiles/configs_bench.py --only ${ONLY:-C3,C4,C5} --reps 5 > $OUT/configs.jsonl 2> $OUT/timing.err
rc=$?
cat $OUT/configs.jsonl; grep "gsdr_trk timing" $OUT/timing.err
exit $rc
