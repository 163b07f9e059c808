#!/usr/bin/env python3
"""A/B sweep of the acquisition correlate-kernel variants (GSDR_ACQ_CORR_VARIANT)
on the bench workload, in one process: per variant the HIP-event time of the
correlate stage and agreement of the per-PRN results with variant 0."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnss-sdr-new_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    import gsdr
    variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,1,2,3,4,5,6".split(","))]
    B = 64
    sats, iq, codes = bench.make_workload(B, 0)
    dev = torch.device("cuda", 0)
    iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    ref = None
    out = {}
    for v in variants:
        os.environ["GSDR_ACQ_CORR_VARIANT"] = str(v)
        acq = gsdr.Acquisition(bench.FS, bench.N, bench.DMAX, bench.DSTEP, pfa=bench.PFA, max_prns=bench.P,
                               max_blocks=B, num_doppler_bins=bench.D)
        acq.set_local_codes(codes, np.arange(1, bench.P + 1))
        res_dev = torch.zeros(B * bench.P * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        for _ in range(30):  # clocks settle
            acq.run_device(iq_dev.data_ptr(), B, bench.N, 0, res_dev.data_ptr(), sptr)
        torch.cuda.synchronize()
        acq.set_profiling(True)
        acq.read_profile()
        for _ in range(30):
            acq.run_device(iq_dev.data_ptr(), B, bench.N, 0, res_dev.data_ptr(), sptr)
        ms, n = acq.read_profile()
        res = res_dev.cpu().numpy().view(gsdr.ACQ_RESULT_DTYPE).reshape(B, bench.P)
        if ref is None:
            ref = res
        same = float(np.mean((res["doppler_index"] == ref["doppler_index"]) & (res["code_phase"] == ref["code_phase"])))
        rel = float(np.max(np.abs(res["test_statistic"] - ref["test_statistic"]) / ref["test_statistic"]))
        out[v] = {"correlate_us": round(ms[1] / n[1] * 1e3, 1), "forward_us": round(ms[0] / n[0] * 1e3, 1),
                  "same_cell_frac": same, "max_stat_rel_diff": rel}
        print(json.dumps({"variant": v, **out[v]}), flush=True)
        acq.close()


if __name__ == "__main__":
    main()
