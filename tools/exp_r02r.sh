#!/bin/bash
# r02r: kernel times and HBM bytes of the C4 acquisition (packed four-step, bit transition)
set -o pipefail
OUT=gpurun_out/r02r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 profiles/configs_bench.py --only C4 --reps 3 > $OUT/c4.jsonl 2> $OUT/c4.err || exit 1
find $OUT/stats -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cut -c1-250 $OUT/kernel_stats.csv | head -12
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 profiles/configs_bench.py --only C4 --reps 2 > /dev/null 2> $OUT/fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 profiles/configs_bench.py --only C4 --reps 2 > /dev/null 2> $OUT/write.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d $OUT/sq -o run --output-format csv -- python3 profiles/configs_bench.py --only C4 --reps 2 > /dev/null 2> $OUT/sq.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/l2 -o run --output-format csv -- python3 profiles/configs_bench.py --only C4 --reps 2 > /dev/null 2> $OUT/l2.err || exit 1
echo done
