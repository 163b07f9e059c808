# Two acquisition chains with a CU partition for the tracking pool.
set -o pipefail
mkdir -p gpurun_out/ch2
for a in "--acq-chains 2 --cu-partition --trk-cus 8" "--acq-chains 2 --cu-partition --trk-cus 4" "--acq-chains 2 --cu-partition --trk-cus 2" "--acq-chains 2" "--acq-chains 2 --cu-partition --trk-cus 16" "--acq-chains 1"; do
  echo "== $a"
  timeout -k 10 120 python bench.py --no-cpu-baseline $a > gpurun_out/ch2/out.json 2>gpurun_out/ch2/err.txt || { tail -5 gpurun_out/ch2/err.txt; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ch2/out.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'),d['check']['acquired_block0'],d['check']['trk_calls_per_channel'])"
done
