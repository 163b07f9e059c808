# Per-phase tracking timing of the last (co-running) launch, two LDS reservations.
set -o pipefail
mkdir -p gpurun_out/tt2
for kb in 156 40; do
  echo "== lds $kb"
  GSDR_TRK_LDS_KB=$kb GSDR_TRK_TIMING=2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/tt2/out.json 2>gpurun_out/tt2/err.txt || { tail -5 gpurun_out/tt2/err.txt; exit 1; }
  grep "gsdr_trk timing" gpurun_out/tt2/err.txt || true
  python -c "import json;d=json.load(open('gpurun_out/tt2/out.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'))"
done
