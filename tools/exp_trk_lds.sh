# Tracking LDS reservation sweep (GSDR_TRK_LDS_KB) on the default bench (co-running with acquisition).
set -o pipefail
mkdir -p gpurun_out/lds
for kb in 40 64 96 128 156 40; do
  echo "== lds $kb KB"
  GSDR_TRK_LDS_KB=$kb timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/lds/out.json 2>gpurun_out/lds/err.txt || { tail -5 gpurun_out/lds/err.txt; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lds/out.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'))"
done
