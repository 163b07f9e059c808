#!/bin/bash
# LDS bank conflicts of the C5 acquisition grids with the default split plans against
# the padded 25000-point row layouts (GSDR_ACQ_SPLIT_ID 7: GPS/BeiDou N = 25000,
# 8: Galileo N = 100000): one SQ counter group, --kernel-trace --stats --pmc only.
#   gpurun -- bash profiles/pmc_c5_pad.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmc_c5_pad}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 cfg=$2 id=$3
  ( if [ -n "$id" ]; then export GSDR_ACQ_SPLIT_ID=$id; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
        SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
        -d "$OUT/${cfg}_$name/sq" -o run --output-format csv -- \
        python3 profiles/acq_cfg_driver.py --cfg $cfg --iters 2 > "$OUT/${cfg}_$name.log" 2>&1 )
}
run base C5g "" && run pad C5g 7 && run base C5e "" && run pad C5e 8 &&
python3 - "$OUT" <<'PY'
import json, os, sys
sys.path.insert(0, "profiles")
from pmc_summary import cfg_json
out = sys.argv[1]
res = {}
for cfg in ("C5g", "C5e"):
    for name in ("base", "pad"):
        for k, v in cfg_json(os.path.join(out, cfg + "_" + name)).items():
            c = v["counters"]
            ia = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
            frac = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / ia if ia else None
            res.setdefault(cfg, {}).setdefault(name, {})[k] = {"avg_us": v.get("avg_us"), "lds_bank_conflict_frac": frac,
                                                               "counters": c}
            print(cfg, name, k[:70], v.get("avg_us"), None if frac is None else round(frac, 4))
json.dump(res, open(os.path.join(out, "pmc_c5_pad.json"), "w"), indent=1)
PY
rc=$?
echo "pmc exit $rc"
exit $rc
