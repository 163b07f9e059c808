#!/bin/bash
# gpu_r06a.sh then gpu_r06b.sh; the second only when the first ended normally (all
# green, rc 0, or a test / check failure, rc 1) -- never after a fault, abort or kill
bash profiles/gpu_r06a.sh "${1:-r06a}"
rc=$?
echo "gpu_r06a exit $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash profiles/gpu_r06b.sh "${2:-r06b}"
