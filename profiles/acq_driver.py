#!/usr/bin/env python3
"""Profiling driver: runs only the C2 acquisition batch (and optionally the
correlator epochs) a fixed number of times, for rocprofv3 kernel-trace / PMC
passes.  Same workload shapes as bench.py."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnss-sdr-new_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--what", choices=["acq", "trk", "both"], default="both")
    a = ap.parse_args()
    import torch
    import gsdr
    from gsdr import synth
    B = a.blocks
    sats, iq, codes = bench.make_workload(B, 0)
    dev = torch.device("cuda", 0)
    iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    res_dev = torch.zeros(B * bench.P * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    trk_out = torch.zeros(bench.CHANNELS * B * gsdr.TRK_EPOCH_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    trk_n = torch.zeros(bench.CHANNELS, dtype=torch.int32, device=dev)
    acq = gsdr.Acquisition(bench.FS, bench.N, bench.DMAX, bench.DSTEP, pfa=bench.PFA, max_prns=bench.P, max_blocks=B,
                           num_doppler_bins=bench.D)
    acq.set_local_codes(codes, np.arange(1, bench.P + 1))
    trk = gsdr.Tracking(bench.trk_conf(bench.CHANNELS))
    for c, s in enumerate(sats):
        delay, dop = bench.acq_result_for(s)
        trk.start(c, s.prn, synth.gps_ca_chips(s.prn), delay, dop, 0, 0)
    trk.save_state(0)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(a.iters):
        if a.what in ("acq", "both"):
            acq.run_device(iq_dev.data_ptr(), B, bench.N, 0, res_dev.data_ptr(), sptr)
        if a.what in ("trk", "both"):
            trk.restore_state(0, sptr)
            trk.run_device(iq_dev.data_ptr(), 0, B * bench.N, B, trk_out.data_ptr(), trk_n.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    trk.close()
    acq.close()
    print("done")


if __name__ == "__main__":
    main()
