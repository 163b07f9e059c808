#!/bin/bash
# the full round pass (gpu_round.sh), then the PPW A/B (gpu_r06h.sh) unless the first
# ended abnormally (anything but a clean exit or a test / check failure)
bash profiles/gpu_round.sh "${1:-r06g}"
rc=$?
echo "gpu_round exit $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash profiles/gpu_r06h.sh "${2:-r06h}"
