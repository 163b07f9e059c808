# kernel timeline of the C2 bench (rocprofv3 --kernel-trace, per-dispatch start/end)
set -o pipefail
OUT=gpurun_out/${1:-r03g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $OUT/timeline.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = None
keep = [r for r in rows if "acq_" in r["Kernel_Name"] or "trk_" in r["Kernel_Name"]]
keep = keep[-90:]
t0 = int(keep[0]["Start_Timestamp"])
for r in keep:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
    print("%10.1f %10.1f %8.1f q%s %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r.get("Queue_Id", r.get("Stream_Id", "?")), name))
PY
cp $f $OUT/kernel_trace.csv
tail -40 $OUT/timeline.txt
