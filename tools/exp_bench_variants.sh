set -o pipefail
mkdir -p gpurun_out/exp1
for a in "" "--only acq" "--only trk" "--blocks 128" "--no-profile-events"; do
  echo "== $a"
  timeout -k 10 120 python bench.py --no-cpu-baseline $a > gpurun_out/exp1/out.json 2>gpurun_out/exp1/err.txt || { tail -5 gpurun_out/exp1/err.txt; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp1/out.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'))"
done
for v in 35 37; do
  echo "== variant $v"
  GSDR_ACQ_CORR_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --only acq > gpurun_out/exp1/out.json 2>gpurun_out/exp1/err.txt || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp1/out.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'))"
done
