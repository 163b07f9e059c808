#!/bin/bash
# One GPU-box pass: parity tests (incl. the host self-test), smoke, the bench line
# (driver flags), rocprofv3 kernel-trace stats of the same bench command, the
# torchrun world-1 path, and the C5 workload line.  Every GPU step has its own
# time limit; the chain stops at the first failure.
#   gpurun --timeout 1100 -- bash profiles/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export GSDR_PARITY_LOG=$OUT/parity_spread.jsonl
rm -f "$GSDR_PARITY_LOG"
echo "== tests" &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1 && tail -3 "$OUT/pytest_gpu.log" &&
grep -E "tracking blocks|channel fsm" "$OUT/pytest_gpu.log" | head -3;
echo "== smoke" &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && cat "$OUT/smoke.log" &&
echo "== bench" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" &&
echo "== rocprof" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench_prof.json" 2> "$OUT/prof.err" &&
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; &&
echo "== torchrun (world size 1, RCCL init + barrier + max-reduce path of bench.py)" &&
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 5 --no-cpu-baseline > "$OUT/bench_torchrun.json" 2> "$OUT/bench_torchrun.err" &&
echo "== c5" &&
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
echo "== configs" &&
timeout -k 10 300 python -u profiles/configs_bench.py --reps 5 > "$OUT/configs.jsonl" 2> "$OUT/configs.err" &&
echo "== receiver (the drop-in path: factory-built pooled tracking blocks + acquisition services, 2 s)" &&
for cfg in c3 c5; do for s in 1 0; do
    timeout -k 10 300 ./gnss-sdr-new_amd/build/receiver_bench $cfg 2 $s > "$OUT/receiver_${cfg}_s$s.json" \
        2> "$OUT/receiver_${cfg}_s$s.err" && cat "$OUT/receiver_${cfg}_s$s.json" || exit 1
done; done
rc=$?
echo "exit $rc"
exit $rc
