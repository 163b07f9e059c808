set -o pipefail
O=gpurun_out/s3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u profiles/sweep_acq_n.py --fs 16000000 --blocks 16 --variants 90,91,92 > $O/sweep16.jsonl 2> $O/sweep16.err && cat $O/sweep16.jsonl &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pa -o run --output-format csv -- python3 profiles/sweep_acq_n.py --fs 16000000 --blocks 16 --variants 90 --reps 2 > $O/pa.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $O/pb -o run --output-format csv -- python3 profiles/sweep_acq_n.py --fs 16000000 --blocks 16 --variants 90 --reps 2 > $O/pb.log 2>&1
echo "exit $?"
