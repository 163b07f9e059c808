#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench line, rocprofv3 kernel-trace stats of
# the same bench command.  Run from the repo root on the GPU box:
#   gpurun --timeout 900 -- bash profiles/gpu_round.sh [tag]
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== tests" &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 && tail -3 "$OUT/pytest_gpu.log" &&
echo "== smoke" &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && cat "$OUT/smoke.log" &&
echo "== bench" &&
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" &&
echo "== rocprof" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 20 > "$OUT/bench_prof.json" 2> "$OUT/prof.err" &&
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; &&
cat "$OUT/kernel_stats.csv" &&
echo "== torchrun (world size 1, RCCL init + barrier + max-reduce path of bench.py)" &&
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 5 --no-cpu-baseline > "$OUT/bench_torchrun.json" 2> "$OUT/bench_torchrun.err" &&
cat "$OUT/bench_torchrun.json"
echo "exit $?"
