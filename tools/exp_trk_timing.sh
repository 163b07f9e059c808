# Per-phase tracking timing (GSDR_TRK_TIMING=2: 100 MHz wall clock ticks) alone and co-running with acquisition.
set -o pipefail
mkdir -p gpurun_out/tt
for a in "--only trk" ""; do
  echo "== $a"
  GSDR_TRK_TIMING=2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 $a > gpurun_out/tt/out.json 2>gpurun_out/tt/err.txt || { tail -5 gpurun_out/tt/err.txt; exit 1; }
  grep "gsdr_trk timing" gpurun_out/tt/err.txt || true
  python -c "import json;d=json.load(open('gpurun_out/tt/out.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'))"
done
