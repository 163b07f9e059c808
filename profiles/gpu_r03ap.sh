#!/bin/bash
# One box: the full round on HEAD (tests, smoke, bench, rocprof, torchrun, C5, configs),
# HEAD's PMC passes, then the tracking per-phase timing.
set -o pipefail
bash profiles/gpu_round.sh r03ap && bash profiles/pmc_r03.sh pmc_r03ap && bash profiles/gpu_trk_timing.sh r03ap_trk notests
