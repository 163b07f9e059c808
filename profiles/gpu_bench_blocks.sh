# C2 bench under the driver's flags (--steps 20 --warmup 5) at several batch sizes
set -o pipefail
OUT=gpurun_out/${1:-r03f}
mkdir -p $OUT
for B in 64 128 256 64; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --blocks $B --no-cpu-baseline > $OUT/bench_b$B.json 2> $OUT/bench_b$B.err || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_b$B.json'));print($B, d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_us_per_launch'], d.get('components'))"
done
for C in 3 4; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --blocks 192 --acq-chains $C --no-cpu-baseline > $OUT/bench_c$C.json 2> $OUT/bench_c$C.err || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_c$C.json'));print('chains', $C, d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
