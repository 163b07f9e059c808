#!/bin/bash
# A/B: tracking workgroup of 512 lanes (default build) vs 256 lanes (build256) in the
# C2 bench (acq + trk co-run), plus the tracking parity tests on the 256-lane build.
set -o pipefail
O=gpurun_out/trk256; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b512_$i.json 2> $O/b512_$i.err || exit 1
  GSDR_LIB=gnss-sdr-new_amd/build256/libgsdr.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b256_$i.json 2> $O/b256_$i.err || exit 1
done
GSDR_LIB=gnss-sdr-new_amd/build256/libgsdr.so timeout -k 10 300 python -u -m pytest tests/test_gpu_trk.py tests/test_gpu_configs.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $O/pytest256.log 2>&1; tail -3 $O/pytest256.log
GSDR_LIB=gnss-sdr-new_amd/build256/libgsdr.so timeout -k 10 200 python -u profiles/configs_bench.py > $O/cfg256.jsonl 2> $O/cfg256.err
python3 - <<'P'
import json
for t in ("b512_1","b256_1","b512_2","b256_2"):
    d=json.load(open("gpurun_out/trk256/%s.json"%t)); print(t, d["value"], d["check"]["channels_within_25hz"], d["stages_us_per_launch"]["trk_loop_all_epochs"])
P
cat $O/cfg256.jsonl
