#!/bin/bash
# r02o: acquisition parity incl. every packed variant; acquisition-only bench per N=4000
# variant; C3 acquisition (N=16000) per variant; PMC (SQ) of variants 31 and 70.
set -o pipefail
OUT=gpurun_out/r02o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_acq.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_acq.log 2>&1
rc=$?; tail -3 $OUT/pytest_acq.log; [ $rc -ne 0 ] && exit $rc
for v in 70 75 76 77 78 31; do
  echo "== variant $v"
  GSDR_ACQ_CORR_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --only acq > $OUT/v$v.json 2> $OUT/v$v.err || { tail -5 $OUT/v$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/v$v.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'))"
done
for v in 60 63; do
  echo "== C3 variant $v"
  GSDR_ACQ_CORR_VARIANT=$v timeout -k 10 200 python profiles/configs_bench.py --only C3 --reps 10 > $OUT/c3_v$v.jsonl 2> $OUT/c3_v$v.err || { tail -5 $OUT/c3_v$v.err; exit 1; }
  grep acquisition $OUT/c3_v$v.jsonl
done
for v in 31 70; do
  GSDR_ACQ_CORR_VARIANT=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $OUT/pmc_sqa_v$v -o run --output-format csv -- python3 profiles/acq_driver.py --iters 2 --what acq > $OUT/pmc_sqa_v$v.log 2>&1 || exit 1
  GSDR_ACQ_CORR_VARIANT=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE -d $OUT/pmc_sqb_v$v -o run --output-format csv -- python3 profiles/acq_driver.py --iters 2 --what acq > $OUT/pmc_sqb_v$v.log 2>&1 || exit 1
done
echo done
