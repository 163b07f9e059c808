#!/bin/bash
# One box: C2 variant A/B (70 vs 71 = 70 at 5 waves per SIMD), then HEAD's PMC passes.
set -o pipefail
bash profiles/gpu_c2_ab.sh r03s 70 71 70 71 && bash profiles/pmc_r03.sh pmc_r03s
