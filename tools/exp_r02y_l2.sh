#!/bin/bash
# Where do the C2 correlate kernel's L2 misses come from?  FETCH_SIZE and TCC hit/miss
# per launch at 32 and 8 PRNs (64 blocks): misses that scale with the PRN count are code
# rows, misses that do not are X rows fetched by several XCDs.
set -o pipefail
O=gpurun_out/l2; mkdir -p $O; export TMPDIR=/tmp
for np in 32 8; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f$np -o run --output-format csv -- python3 profiles/sweep_acq_n.py --fs 4000000 --blocks 64 --variants 70 --reps 2 --prns $np > $O/f$np.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $O/t$np -o run --output-format csv -- python3 profiles/sweep_acq_n.py --fs 4000000 --blocks 64 --variants 70 --reps 2 --prns $np > $O/t$np.log 2>&1 || exit 1
done
python3 - <<'P'
import csv,collections,glob
for d in ("f32","t32","f8","t8"):
    agg=collections.defaultdict(float); n=collections.Counter()
    for f in glob.glob("gpurun_out/l2/%s/**/*counter_collection.csv"%d, recursive=True):
        for r in csv.DictReader(open(f)):
            if "acq_correlate" in r["Kernel_Name"]:
                agg[r["Counter_Name"]]+=float(r["Counter_Value"]); n[r["Counter_Name"]]+=1
    print(d, {k: v/n[k] for k,v in agg.items()})
P
