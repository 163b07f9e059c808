#!/bin/bash
# Round 6: the multi-rank bench path on real engines, two ranks sharing the box's one GPU
# (GSDR_BENCH_SHARED_DEVICE=1, gloo collectives): the GPU test, then the C2 and C5 lines at
# world 2 for the record (a rehearsal, not a scaling number).
set -o pipefail
TAG=${1:-r06m}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v -s --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_multirank.log" 2>&1; rc=$?; tail -5 "$OUT/pytest_multirank.log"; [ $rc -eq 0 ] || exit $rc
export GSDR_BENCH_SHARED_DEVICE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_c2_world2.json" 2> "$OUT/bench_c2_world2.err" || exit 1
cut -c1-400 "$OUT/bench_c2_world2.json"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
    bench.py --workload c5 --gpus 2 --steps 10 --warmup 3 > "$OUT/bench_c5_world2.json" 2> "$OUT/bench_c5_world2.err" || exit 1
cut -c1-400 "$OUT/bench_c5_world2.json"
