#!/bin/bash
# One box: the full round (tests, smoke, bench, rocprof, torchrun, C5, configs), then the
# tracking per-phase timing (incl. the streamed correlation's stream-wait share).
set -o pipefail
bash profiles/gpu_round.sh r03u && bash profiles/gpu_trk_timing.sh r03u_trk notests
