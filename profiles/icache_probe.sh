#!/bin/bash
# Instruction-cache counters over the tracking-only bench (C2): lists the gfx950 counters,
# then one --pmc pass with the SQC instruction-cache counters if the list has them.
#   gpurun -- bash profiles/icache_probe.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r03ac}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || { echo "list failed"; exit 1; }
grep -oE "SQC_ICACHE_[A-Z_]+|SQ_IFETCH[A-Z_]*|SQ_INSTS_VALU\b|SQ_WAIT_INST_ANY|SQ_BUSY_CYCLES|SQ_WAVE_CYCLES" "$OUT/counters_list.txt" | sort -u > "$OUT/icache_names.txt"
cat "$OUT/icache_names.txt"
grep -q "SQC_ICACHE_MISSES$" "$OUT/icache_names.txt" || grep -q "SQC_ICACHE_MISSES" "$OUT/icache_names.txt" || exit 0
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
    -d "$OUT/pmc_ic" -o pmc --output-format csv -- python3 bench.py --only trk --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/pmc_ic.log" 2>&1
rc=$?; tail -2 "$OUT/pmc_ic.log"; exit $rc
