#!/bin/bash
# Round 6 evidence pass on HEAD: the full round pass (tests, smoke, bench, rocprof,
# torchrun world 1, C5 line, configurations, receiver), then the rocFFT A/B, the PMC
# passes and the receiver kernel trace -- each only after the previous ended cleanly.
set -o pipefail
TAG=${1:-r06d}
bash profiles/gpu_round.sh "$TAG" || exit $?
echo "== rocFFT A/B" &&
timeout -k 10 300 ./gnss-sdr-new_amd/build/rocfft_ab 5 > "gpurun_out/$TAG/rocfft_ab.jsonl" 2> "gpurun_out/$TAG/rocfft_ab.err" &&
cat "gpurun_out/$TAG/rocfft_ab.jsonl" &&
bash profiles/gpu_r06c.sh "$TAG/c"
