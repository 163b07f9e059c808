#!/bin/bash
# Round 6: PRN-group size of the split grids (code bytes per XCD pass, GSDR_ACQ_GROUP_KB) A/B.
set -o pipefail
bash profiles/ab_sweep.sh "${1:-r06g2}" "python -u profiles/configs_bench.py --only C5 --acq-only --reps 5" \
    "GSDR_ACQ_GROUP_KB=2048" "GSDR_ACQ_GROUP_KB=512" "GSDR_ACQ_GROUP_KB=1024" "GSDR_ACQ_GROUP_KB=4096" "GSDR_ACQ_GROUP_KB=8192" "GSDR_ACQ_GROUP_KB=2048"
