#!/bin/bash
# General-path (dwells / bit transition) parity after the XCD-aware dwell grid, and the C4 line.
set -o pipefail
O=gpurun_out/c4xcd; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_acq_dwells.py tests/test_gpu_acq_signals.py tests/test_gpu_acq_two_step.py tests/test_gpu_acq.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; tail -3 $O/pytest.log
timeout -k 10 200 python -u profiles/configs_bench.py --only C4 > $O/c4.jsonl 2> $O/c4.err; cat $O/c4.jsonl
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f -o run --output-format csv -- python3 profiles/acq_cfg_driver.py --cfg C4 --iters 2 > $O/f.log 2>&1
timeout -k 10 200 python -u profiles/sweep_acq_n.py --fs 4000000 --blocks 64 --variants 70,79,80,78,70,79,80 > $O/sweep4.jsonl 2> $O/sweep4.err; cat $O/sweep4.jsonl
