#!/bin/bash
# Kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes of the C3 and C4 acquisitions.
set -o pipefail
O=gpurun_out/pmc_cfg; mkdir -p $O; export TMPDIR=/tmp
for c in C3 C4; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/${c}_t -o run --output-format csv -- python3 profiles/acq_cfg_driver.py --cfg $c --iters 4 > $O/${c}_t.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/${c}_f -o run --output-format csv -- python3 profiles/acq_cfg_driver.py --cfg $c --iters 2 > $O/${c}_f.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/${c}_w -o run --output-format csv -- python3 profiles/acq_cfg_driver.py --cfg $c --iters 2 > $O/${c}_w.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d $O/${c}_s -o run --output-format csv -- python3 profiles/acq_cfg_driver.py --cfg $c --iters 2 > $O/${c}_s.log 2>&1 || exit 1
done
echo "pmc ok"
