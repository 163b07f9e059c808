#!/usr/bin/env python3
"""Micro-benchmark of the tracking correlator launch (bench workload shapes):
device job table (run_epochs / run_batch_device, rotator model on the device)
vs host job table (run_batch, rotator model from the host), per-launch kernel time."""
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
    from gsdr import synth
    B = 64
    sats, iq, codes, jobs = bench.make_workload(B, 0)
    dev = torch.device("cuda", 0)
    iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    jobs_dev = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    out = torch.zeros(B * bench.CHANNELS * bench.TAPS * 2, dtype=torch.float32, device=dev)
    corr = gsdr.Correlator(bench.CHANNELS * B, bench.N, max_taps=bench.TAPS)
    for c, s in enumerate(sats):
        corr.set_local_code_and_taps(c, synth.gps_ca_chips(s.prn), np.array([-0.5, 0.0, 0.5], np.float32))
    sptr = torch.cuda.current_stream(dev).cuda_stream
    res = {}
    for name in ("epochs_device_jobs", "batch_host_jobs_per_epoch", "one_launch_all_jobs"):
        for rep in range(2):
            corr.set_profiling(True)
            corr.read_profile()
            if name == "epochs_device_jobs":
                corr.run_epochs(jobs_dev.data_ptr(), bench.CHANNELS, B, iq_dev.data_ptr(), B * bench.N,
                                out.data_ptr(), stream_ptr=sptr)
            elif name == "batch_host_jobs_per_epoch":
                for e in range(B):
                    corr.run_batch(jobs[e * bench.CHANNELS:(e + 1) * bench.CHANNELS], iq_dev.data_ptr(),
                                   B * bench.N, out.data_ptr(), stream_ptr=sptr)
            else:
                corr.run_batch(jobs, iq_dev.data_ptr(), B * bench.N, out.data_ptr(), stream_ptr=sptr)
            torch.cuda.synchronize()
            ms, n = corr.read_profile()
        res[name] = {"launches": n, "us_per_launch": round(ms / n * 1e3, 2)}
        print(json.dumps({name: res[name]}), flush=True)


if __name__ == "__main__":
    main()
