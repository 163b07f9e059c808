#!/usr/bin/env python3
"""Profiling driver for the large-N acquisition configurations only (no tracking),
same shapes as configs_bench.py: C3 = GPS 16 Msps, N = 16000, 32 PRN x 81 Doppler,
16 blocks per call; C4 = Galileo E1 8 Msps, bit transition (FFT 64000), 36 PRN x 81
Doppler, 4 blocks per call.  Runs --iters calls, for rocprofv3 kernel-trace / PMC
passes."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnss-sdr-new_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", choices=["C3", "C4", "C4s", "C5g", "C5e"], default="C3")
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import torch
    import gsdr
    from gsdr import synth
    dev = torch.device("cuda", 0)
    if a.cfg == "C3":
        fs, N, B = 16000000, 16000, 16
        sats = synth.random_constellation(12, seed_offset=3, prns=list(range(1, 13)))
        iq = synth.gps_l1_iq(fs, B * N, sats, seed_offset=3)
        acq = gsdr.Acquisition(fs, N, 10000, 250, pfa=0.01, max_prns=32, max_blocks=B, num_doppler_bins=81)
        acq.set_local_codes(np.stack([synth.gps_ca_sampled(p, fs) for p in range(1, 33)]), np.arange(1, 33))
        P, n_call = 32, N
    elif a.cfg == "C4s":  # C4 without bit transition: one 4 ms period, FFT 32000
        fs, N, B = 8000000, 32000, 4
        rng = np.random.default_rng(4)
        gsats = [synth.GalileoSatellite(p, float(rng.uniform(-4000, 4000)), float(rng.uniform(0, 4092)), 46.0,
                                        float(rng.uniform(0, 6.28))) for p in range(1, 9)]
        iq = synth.gal_e1_iq(fs, B * N + N, gsats, seed_offset=4)
        acq = gsdr.Acquisition(fs, N, 5000, 125, pfa=0.0, max_prns=36, max_blocks=B, sampled_ms=4, ms_per_code=4)
        codes = np.stack([synth.gal_e1_sampled(p, fs, pilot=True)[:N] for p in range(1, 37)])
        acq.set_local_codes(codes, np.arange(1, 37))
        acq.set_threshold(2.5)
        P, n_call = 36, N
    elif a.cfg in ("C5g", "C5e"):  # one GPU's C5 share: GPS N = 25000 / Galileo N = 100000
        fs, B = 25000000, 4
        N = 25000 if a.cfg == "C5g" else 100000
        sats = synth.random_constellation(8, seed_offset=5, prns=list(range(1, 9)))
        iq = synth.gps_l1_iq(fs, B * N + N, sats, seed_offset=5)
        ms = N // 25000
        P = 32 if a.cfg == "C5g" else 36
        acq = gsdr.Acquisition(fs, N, 10000 if ms == 1 else 5000, 250, pfa=0.01, max_prns=P, max_blocks=B,
                               sampled_ms=ms, ms_per_code=ms)
        if a.cfg == "C5g":
            codes = np.stack([synth.gps_ca_sampled(p, fs) for p in range(1, 33)])
        else:
            codes = np.stack([synth.gal_e1_sampled(p, fs, pilot=True)[:N] for p in range(1, 37)])
        acq.set_local_codes(codes, np.arange(1, P + 1))
        n_call = N
    else:
        fs, N, B = 8000000, 32000, 4
        rng = np.random.default_rng(4)
        gsats = [synth.GalileoSatellite(p, float(rng.uniform(-4000, 4000)), float(rng.uniform(0, 4092)), 46.0,
                                        float(rng.uniform(0, 6.28))) for p in range(1, 9)]
        iq = synth.gal_e1_iq(fs, B * 2 * N + 2 * N, gsats, seed_offset=4)
        acq = gsdr.Acquisition(fs, 2 * N, 5000, 125, pfa=0.0, max_prns=36, max_blocks=B, sampled_ms=4,
                               ms_per_code=4, bit_transition=True)
        codes = np.stack([np.resize(synth.gal_e1_sampled(p, fs, pilot=True), 2 * N) for p in range(1, 37)])
        acq.set_local_codes(codes, np.arange(1, 37))
        acq.set_threshold(2.5)
        P, n_call = 36, 2 * N
    iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    res = torch.zeros(B * P * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    for _ in range(a.iters):
        acq.run_device(iq_dev.data_ptr(), B, n_call, 0, res.data_ptr())
    torch.cuda.synchronize()
    acq.close()
    print("done", a.cfg, a.iters)


if __name__ == "__main__":
    main()
