set -o pipefail
OUT=gpurun_out/r03e
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
rc=$?; cat $OUT/bench_c5.json; tail -3 $OUT/bench_c5.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --workload c5 --gpus 1 --steps 5 --warmup 2 > $OUT/bench_c5_torchrun.json 2> $OUT/bench_c5_torchrun.err
rc=$?; cat $OUT/bench_c5_torchrun.json; exit $rc
