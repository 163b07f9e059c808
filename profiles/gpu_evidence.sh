#!/bin/bash
# ${TAG}: round-4 evidence on HEAD: the full round (tests, smoke, bench with CPU
# baseline, rocprof stats, torchrun world 1, C5 stream line, config lines), HEAD's PMC
# passes (bench traffic source), and the drop-in receiver path at C3 / C5 scale with
# and without the acquisition services' searches.
set -o pipefail
TAG=${1:-r04k}
bash profiles/gpu_round.sh ${TAG} && bash profiles/pmc_r03.sh pmc_${TAG} || exit $?
OUT=gpurun_out/${TAG}
for spec in "c3 0.4 0" "c3 0.4 1" "c5 0.4 0" "c5 0.4 1"; do
  set -- $spec
  echo "== receiver_bench $spec"
  timeout -k 10 240 ./gnss-sdr-new_amd/build/receiver_bench $1 $2 $3 > "$OUT/receiver_$1_s$3.json" \
      2> "$OUT/receiver_$1_s$3.err" || exit $?
  cat "$OUT/receiver_$1_s$3.json"
done
