#!/bin/bash
set -o pipefail
O=gpurun_out/full; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; tail -3 $O/pytest.log
timeout -k 10 300 python -u profiles/configs_bench.py > $O/configs.jsonl 2> $O/configs.err; cat $O/configs.jsonl; tail -3 $O/configs.err
