# Acquisition split over several handles/streams (pipelined forward and correlate).
set -o pipefail
mkdir -p gpurun_out/ch
for a in "--acq-chains 1" "--acq-chains 2" "--acq-chains 4" "--acq-chains 2 --only acq" "--acq-chains 1 --only acq" "--acq-chains 1" "--acq-chains 2"; do
  echo "== $a"
  timeout -k 10 120 python bench.py --no-cpu-baseline $a > gpurun_out/ch/out.json 2>gpurun_out/ch/err.txt || { tail -5 gpurun_out/ch/err.txt; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ch/out.json'));print(d['value'],d['ms_per_step'],d.get('stages_us_per_launch'),d['check']['acquired_block0'])"
done
