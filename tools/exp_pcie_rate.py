"""PCIe-inclusive rate of the synchronous host boundary (gsdr_acq_run).

The bench's `value` is measured with the IQ already resident in HBM (gsdr_acq_run_device).
A GNSS-SDR block calling the drop-in through `gsdr_acq_run` hands over a HOST buffer: the
call copies the blocks host->device, runs the same grid and copies the results back.  This
script times that path on the bench's C2 acquisition workload (4 Msps, 32 PRN x 81 Doppler,
64 blocks of 1 ms per call) next to the device-resident rate, for pageable and pinned host
input, and prints one JSON line.  Acquisition only; tracking is not part of this boundary.

    python tools/exp_pcie_rate.py [--calls 20] [--blocks 64]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnss-sdr-new_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (workload constants and synthetic capture)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=64)
    args = ap.parse_args()

    import torch
    import gsdr

    B, K = args.blocks, args.calls
    _, iq, codes = bench.make_workload(B, 0)
    iq = np.ascontiguousarray(iq, np.complex64)
    a = gsdr.Acquisition(bench.FS, bench.N, bench.DMAX, bench.DSTEP, pfa=bench.PFA, max_prns=bench.P,
                         max_blocks=B, num_doppler_bins=bench.D, device=0)
    a.set_local_codes(codes, np.arange(1, bench.P + 1))
    samples = B * bench.N

    def rate_host(buf):
        for _ in range(args.warmup):
            a.run(buf, nblocks=B)
        t0 = time.perf_counter()
        for _ in range(K):
            out = a.run(buf, nblocks=B)
        dt = (time.perf_counter() - t0) / K
        return samples / dt / 1e6, dt * 1e3, out

    r_pageable, ms_pageable, out_h = rate_host(iq)

    pinned = torch.from_numpy(iq.view(np.float32).copy()).pin_memory()
    iq_pinned = pinned.numpy().view(np.complex64)
    r_pinned, ms_pinned, _ = rate_host(iq_pinned)

    dev = torch.device("cuda", 0)
    iq_dev = pinned.to(dev)
    res_dev = torch.zeros(B * bench.P * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    for _ in range(args.warmup):
        a.run_device(iq_dev.data_ptr(), B, bench.N, 0, res_dev.data_ptr())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        a.run_device(iq_dev.data_ptr(), B, bench.N, 0, res_dev.data_ptr())
    torch.cuda.synchronize()
    dt_dev = (time.perf_counter() - t0) / K
    out_d = np.frombuffer(res_dev.cpu().numpy().tobytes(), gsdr.ACQ_RESULT_DTYPE).reshape(B, bench.P)

    same = bool(all(np.array_equal(out_h[f], out_d[f])
                    for f in ("code_phase", "doppler_index", "test_statistic", "positive")))
    h2d_gbs = samples * 8 / (ms_pinned * 1e-3) / 1e9
    print(json.dumps({
        "what": "gsdr_acq_run (host buffer, PCIe-inclusive) vs gsdr_acq_run_device (HBM-resident)",
        "workload": f"C2 acquisition: {B} x 1 ms blocks, 4 Msps gr_complex, {bench.P} PRN x {bench.D} Doppler, one handle",
        "host_pageable_msps": round(r_pageable, 2), "host_pageable_ms_per_call": round(ms_pageable, 3),
        "host_pinned_msps": round(r_pinned, 2), "host_pinned_ms_per_call": round(ms_pinned, 3),
        "device_resident_msps": round(samples / dt_dev / 1e6, 2), "device_ms_per_call": round(dt_dev * 1e3, 3),
        "input_bytes_per_call": samples * 8, "pinned_effective_GBps_incl_compute": round(h2d_gbs, 2),
        "host_and_device_results_identical": same,
    }))


if __name__ == "__main__":
    main()
