# Correlate-variant sweep on the bench workload (acquisition only), one bench per variant.
set -o pipefail
mkdir -p gpurun_out/expv
for v in ${VARIANTS:-30 31 32 33}; do
  echo "== variant $v"
  GSDR_ACQ_CORR_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --only acq > gpurun_out/expv/out.json 2>gpurun_out/expv/err.txt || { tail -5 gpurun_out/expv/err.txt; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/expv/out.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'))"
done
