#!/usr/bin/env python3
"""A/B sweep of the packed correlate variants (GSDR_ACQ_CORR_VARIANT) at any
1 ms FFT size: 32 PRN x 81 Doppler over B blocks of a synthetic GPS stream, per
variant the HIP-event stage times (forward, correlate, reduce + argmax) and the
agreement of the per-PRN results with the first variant listed.

  python profiles/sweep_acq_n.py --fs 16000000 --blocks 16 --variants 60,63,66,67
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnss-sdr-new_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fs", type=int, default=16000000)
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--variants", default="60,63")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--prns", type=int, default=32)
    a = ap.parse_args()
    import torch
    import gsdr
    from gsdr import synth
    fs, B = a.fs, a.blocks
    N = fs // 1000
    sats = synth.random_constellation(8, seed_offset=3, prns=list(range(1, 9)))
    iq = synth.gps_l1_iq(fs, B * N, sats, seed_offset=3)
    NP = a.prns
    codes = np.stack([synth.gps_ca_sampled(p, fs) for p in range(1, NP + 1)])
    dev = torch.device("cuda", 0)
    iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    ref = None
    for v in [int(x) for x in a.variants.split(",")]:
        os.environ["GSDR_ACQ_CORR_VARIANT"] = str(v)
        acq = gsdr.Acquisition(fs, N, 10000, 250, pfa=0.01, max_prns=NP, max_blocks=B, num_doppler_bins=81)
        acq.set_local_codes(codes, np.arange(1, NP + 1))
        res_dev = torch.zeros(B * NP * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        for _ in range(5):
            acq.run_device(iq_dev.data_ptr(), B, N, 0, res_dev.data_ptr(), sptr)
        torch.cuda.synchronize()
        acq.set_profiling(True)
        acq.read_profile()
        for _ in range(a.reps):
            acq.run_device(iq_dev.data_ptr(), B, N, 0, res_dev.data_ptr(), sptr)
        torch.cuda.synchronize()
        ms, n = acq.read_profile()
        acq.set_profiling(False)
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.reps):
            acq.run_device(iq_dev.data_ptr(), B, N, 0, res_dev.data_ptr(), sptr)
        t1.record()
        torch.cuda.synchronize()
        wall = t0.elapsed_time(t1) / a.reps
        res = res_dev.cpu().numpy().view(gsdr.ACQ_RESULT_DTYPE).reshape(B, NP)
        if ref is None:
            ref = res
        same = float(np.mean((res["doppler_index"] == ref["doppler_index"]) & (res["code_phase"] == ref["code_phase"])))
        rel = float(np.max(np.abs(res["test_statistic"] - ref["test_statistic"]) / ref["test_statistic"]))
        st = {k: round(float(ms[i] / max(1, n[i]) * 1e3), 1) for i, k in enumerate(("forward_us", "correlate_us", "reduce_us", "second_us"))}
        print(json.dumps({"variant": v, "N": N, "blocks": B, **st, "ms_per_call": round(wall, 4),
                          "msps": round(B * N / wall / 1e3, 2), "same_cell_frac": same,
                          "max_stat_rel_diff": rel}), flush=True)
        acq.close()


if __name__ == "__main__":
    main()
