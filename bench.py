#!/usr/bin/env python3
"""Benchmark: IQ Msamples/s processed (acquisition + tracking) on BASELINE config C2.

One step = one batch of B consecutive 1 ms blocks of synthetic GPS L1 C/A IQ at
4 Msps already resident in HBM; over the batch:
  - a full PCPS acquisition grid per block: 32 PRNs x 81 Doppler bins (+-10 kHz,
    250 Hz), CFAR (pfa 0.01) -- pcps_acquisition::acquisition_core for all PRNs;
  - closed-loop DLL/PLL tracking of the 8 visible satellites over the same span:
    every general_work call of dll_pll_veml_tracking (3-tap E-P-L correlation of
    4000 samples + discriminators + loop filters + NCO update + lock detectors),
    device-resident (gsdr_trk_run_device), the channel state restored to the same
    start each step so every step re-tracks the same 64 ms.
Acquisition and tracking run on separate HIP streams (they are independent work):
the acquisition blocks of a step are split over two handles (--acq-chains 2), so one
chain's forward-spectra kernel overlaps the other's correlate grid.
Whole-job throughput = blocks * 4000 samples * ranks / max-over-ranks wall time.

Multi-GPU: one process per GPU (torch.distributed.run); every rank processes its
own independent stream shard (weak scaling, no data-path collective).

Also reports: the dominant kernel's roofline (algorithmic bytes / average launch
time from HIP events recorded on the launch stream) and a CPU baseline (the
oracle restatement, timed on this host on a bounded sample, rank 0 at N=1 only).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gnss-sdr-new_amd"))
sys.path.insert(0, ROOT)

METRIC = "IQ Msamples/s processed (acq+track), 32 PRN × 81 Doppler; % HBM roofline"
FS = 4000000
N = 4000               # samples per 1 ms block (consumed_samples = fft_size)
P = 32                 # PRNs searched per block
D = 81                 # Doppler bins (inclusive +-10 kHz grid at 250 Hz)
DMAX, DSTEP = 10000, 250
PFA = 0.01
CHANNELS = 8           # tracked satellites
TAPS = 3               # E, P, L
HBM_PEAK = 8.0e12      # MI355X HBM3E spec (MI355X_MICROARCH.md)


def acq_bytes_per_block():
    """B_acq = 8N(1 + D + P*D) + 16*P*D per N-sample block."""
    return 8 * N * (1 + D + P * D) + 16 * P * D


def correlate_kernel_bytes_per_block():
    """Dominant kernel's share: each P*D cell streams its N-point spectrum once (8N)
    and writes a 16-byte row-statistics tuple."""
    return 8 * N * P * D + 16 * P * D


def trk_bytes_per_epoch():
    """B_trk = 8N + 8K per channel-epoch."""
    return 8 * N + 8 * TAPS


def acq_result_for(s):
    """What acquisition reports for satellite s at stamp 0: code-start sample, grid Doppler."""
    tau = s.code_delay_chips / 1.023e6 * FS
    return float(round(tau) % N), float(DSTEP * round(s.doppler_hz / DSTEP))


def trk_conf(nch):
    import gsdr
    c = gsdr.trk_conf_default()
    c["fs_in"] = FS
    c["pll_bw_hz"] = 40.0   # conf/gnss-sdr_GPS_L1_gr_complex.conf:66-67
    c["dll_bw_hz"] = 4.0
    c["max_channels"] = nch
    return c


def make_workload(blocks, rank, periodic=False):
    from gsdr import synth
    sats = synth.random_constellation(CHANNELS, seed_offset=100 + rank)
    if periodic:
        # a whole number of carrier cycles per batch: the batch repeated end to end
        # is a continuous signal (the code has 1 ms period and no code Doppler here)
        span = blocks * N / FS
        for s in sats:
            s.doppler_hz = round(s.doppler_hz * span) / span
    iq = synth.gps_l1_iq(FS, blocks * N, sats, seed_offset=100 + rank)
    codes = np.stack([synth.gps_ca_sampled(p, FS) for p in range(1, P + 1)])
    return sats, iq, codes


def cpu_baseline(iq, codes, sats, budget_s=12.0):
    """Oracle restatement on this host's CPU (1 thread): numpy pocketfft complex64
    PCPS (acquisition_core + CFAR statistic) for all 32 PRNs x 81 bins of a block,
    plus the C restatement of dll_pll_veml_tracking (generic VOLK correlator + loop)
    for every channel's general_work call in the block."""
    from oracle import pcps, trk
    from gsdr import synth
    wipe = pcps.doppler_wipeoffs(FS, N, DMAX, DSTEP, D)
    cconj = np.conj(np.fft.fft(codes.astype(np.complex64), axis=1)).astype(np.complex64)
    chans = []
    for s in sats:
        o = trk.Channel(trk_conf(1).view(trk.TRK_CONF_DTYPE))
        delay, dop = acq_result_for(s)
        first = o.start(synth.gps_ca_chips(s.prn), delay, dop, 0, 0)
        chans.append([o, first])
    rec = np.zeros(1, trk.TRK_EPOCH_DTYPE)
    L = trk._lib()

    def one_block(b):
        x = iq[b * N:(b + 1) * N]
        X = np.fft.fft(x[None, :] * wipe, axis=1).astype(np.complex64)
        for p in range(P):
            R = np.fft.ifft(X * cconj[p][None, :], axis=1) * N
            M = (R.real * R.real + R.imag * R.imag).astype(np.float32)
            pcps.max_to_input_power_statistic(M)
        for c in chans:
            o, n = c
            if n + N <= len(iq):
                L.orc_trk_call(o._h, iq[n:].ctypes.data, n, rec.ctypes.data)
                c[1] = n + int(rec["consumed"][0])

    t0 = time.perf_counter()
    one_block(0)
    t1 = time.perf_counter() - t0
    nblk = int(max(1, min(len(iq) // N - 1, math.ceil(budget_s / max(t1, 1e-3)))))
    t0 = time.perf_counter()
    for b in range(1, nblk + 1):
        one_block(b)
    dt = time.perf_counter() - t0
    return {"value": round(nblk * N / dt / 1e6, 5), "unit": "Msamples/s", "cores": 1, "kind": "port",
            "sample": "%d blocks of 1 ms (4000 samples): 32 PRN x 81 Doppler CFAR PCPS (numpy pocketfft complex64) "
                      "+ one dll_pll_veml_tracking call (C restatement: generic VOLK 3-tap correlator + DLL/PLL) "
                      "for each of 8 channels; %.1f s on one host core" % (nblk, dt)}


def load_pmc_traffic():
    """HBM bytes per launch of the dominant kernel, from the committed rocprofv3 PMC
    summary (profiles/pmc_*.json, written by profiles/collect_pmc.py), if present."""
    best = None
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    for f in sorted(os.listdir(pdir)):
        if f.startswith("pmc_") and f.endswith(".json"):
            try:
                d = json.load(open(os.path.join(pdir, f)))
                best = d
            except Exception:
                pass
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=64, help="1 ms blocks per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile-events", action="store_true")
    ap.add_argument("--cu-partition", action="store_true",
                    help="give the tracking stream CHANNELS CUs of its own and acquisition the rest")
    ap.add_argument("--trk-cus", type=int, default=0,
                    help="with --cu-partition: CUs reserved for tracking (default: one per channel)")
    ap.add_argument("--acq-chains", type=int, default=2,
                    help="split the step's blocks over this many acquisition handles, each on its own stream "
                         "(2: one chain's forward spectra overlap the other's correlate grid; at most 3 with the "
                         "tracking stream, GPU_MAX_HW_QUEUES = 4)")
    ap.add_argument("--trk-stream", action="store_true",
                    help="tracking follows one continuous stream (the batch repeated, Dopplers on whole cycles per "
                         "batch): one tracking launch covers all timed steps instead of one launch per step")
    ap.add_argument("--only", choices=["acq", "trk"], default=None,
                    help="diagnostic: run only one of the two stages (the line is then not the metric)")
    args = ap.parse_args()

    import torch
    import gsdr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B = args.blocks

    sats, iq, codes = make_workload(B, rank, periodic=args.trk_stream)
    iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    res_dev = torch.zeros(B * P * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    W, K = args.warmup, args.steps
    if args.trk_stream:
        # the tracking stream: warmup + timed batches end to end
        iq_long = iq_dev.repeat(W + K + 1)  # + one batch of slack for the last calls
        trk_epochs = max(W, K) * B
    else:
        iq_long = iq_dev
        trk_epochs = B
    trk_out = torch.zeros(CHANNELS * trk_epochs * gsdr.TRK_EPOCH_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    trk_n = torch.zeros(CHANNELS, dtype=torch.int32, device=dev)

    nch = max(1, args.acq_chains)
    assert B % nch == 0, "--blocks must be a multiple of --acq-chains"
    Bc = B // nch
    acqs = []
    for _ in range(nch):
        a = gsdr.Acquisition(FS, N, DMAX, DSTEP, pfa=PFA, max_prns=P, max_blocks=Bc, num_doppler_bins=D,
                             device=local)
        a.set_local_codes(codes, np.arange(1, P + 1))
        acqs.append(a)
    acq = acqs[0]
    trk = gsdr.Tracking(trk_conf(CHANNELS), device=local)
    from gsdr import synth
    for c, s in enumerate(sats):
        delay, dop = acq_result_for(s)
        trk.start(c, s.prn, synth.gps_ca_chips(s.prn), delay, dop, 0, 0)
    # each handle launches on its own HIP stream (its own hardware queue).  The
    # tracking pool is a latency chain of one workgroup per channel that needs a
    # whole CU; give it CHANNELS CUs (one per XCD for 8) and the acquisition grid
    # the other 248, so neither waits for the other's workgroups to drain.
    if args.cu_partition:
        trk_mask, acq_mask = gsdr.cu_partition(args.trk_cus or CHANNELS)
        trk.set_cu_mask(trk_mask)
        for a in acqs:
            a.set_cu_mask(acq_mask)
    trk.save_state(0)

    def trk_stream_launch(nsteps):
        # one launch: nsteps * B general_work calls per channel, continuing the stream
        if args.only != "acq" and nsteps > 0:
            trk.run_device(iq_long.data_ptr(), 0, (W + K + 1) * B * N, nsteps * B, trk_out.data_ptr(), trk_n.data_ptr())

    def step():
        if args.only != "acq" and not args.trk_stream:
            trk.restore_state(0)
            trk.run_device(iq_dev.data_ptr(), 0, B * N, B, trk_out.data_ptr(), trk_n.data_ptr())
        if args.only != "trk":
            for i, a in enumerate(acqs):
                a.run_device(iq_dev.data_ptr() + i * Bc * N * 8, Bc, N, i * Bc * N,
                             res_dev.data_ptr() + i * Bc * P * gsdr.ACQ_RESULT_DTYPE.itemsize)

    if args.trk_stream:
        trk_stream_launch(W)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # sanity: the visible satellites are acquired and tracked with a strong prompt
    res = res_dev.cpu().numpy().view(gsdr.ACQ_RESULT_DTYPE).reshape(B, P)
    det = {int(r["prn"]) for r in res[0] if r["positive"]}
    vis = {s.prn for s in sats}
    ep_warm = max(W * B, 1) if args.trk_stream else B  # the warmup launch's max_epochs (record layout)
    recs = trk_out.cpu().numpy().view(gsdr.TRK_EPOCH_DTYPE)[:CHANNELS * ep_warm].reshape(CHANNELS, ep_warm)
    nrec = trk_n.cpu().numpy()
    taps = np.stack([recs[c][nrec[c] - 1]["taps"][:6].view(np.complex64) for c in range(CHANNELS)])
    prompt_ratio = float(np.median(np.abs(taps[:, 1]) / np.maximum(np.abs(taps[:, 0]), 1e-9)))
    # carrier Doppler averaged over the last 16 calls (one call's value carries the
    # PLL's per-epoch jitter at 40 Hz loop bandwidth); channels start from the
    # 250 Hz acquisition grid, so some are still pulling in after 64 ms
    dop_err = np.array([abs(np.mean(recs[c][max(nrec[c] - 16, 0):nrec[c]]["carrier_doppler_hz"]) - sats[c].doppler_hz)
                        for c in range(CHANNELS)]) if nrec.min() > 0 else None

    if not args.no_profile_events:
        for a in acqs:
            a.set_profiling(True)
            a.read_profile()
        trk.set_profiling(True)
        trk.read_profile()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if args.trk_stream:
        trk_stream_launch(K)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    trk_calls_timed = int(trk_n.cpu().numpy().min())
    stage_ms, stage_n = (np.zeros(4), np.zeros(4, np.uint32))
    trk_ms, trk_launches = 0.0, 0
    if not args.no_profile_events:
        for a in acqs:
            ms_a, n_a = a.read_profile()
            stage_ms = stage_ms + ms_a
            stage_n = stage_n + n_a
        trk_ms, trk_launches = trk.read_profile()

    samples = world * args.steps * B * N
    value = samples / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded GPS L1 C/A IQ, 8 visible PRNs at 45 dB-Hz + AWGN, per-rank shard)",
        "config": {
            "workload": "C2: GPS L1 C/A 4 Msps; per 1 ms block a 32 PRN x 81 Doppler (+-10 kHz, 250 Hz) CFAR PCPS "
                        "grid + closed-loop DLL/PLL tracking (3-tap E-P-L, dll_pll_veml_tracking) of 8 channels "
                        "over the same span",
            "blocks_per_step": B, "fs_sps": FS, "fft_size": N, "prns": P, "doppler_bins": D, "channels": CHANNELS,
            "taps": TAPS, "item_type": "gr_complex", "parallelism": "blocks sharded per rank (dp%d)" % world,
            "tracking": ("one continuous stream, one launch per timed region" if args.trk_stream
                         else "64 ms re-tracked per step from a saved state, one launch per step"),
            "cu_partition": ({"tracking": args.trk_cus or CHANNELS, "acquisition": 256 - (args.trk_cus or CHANNELS)}
                             if args.cu_partition else None),
            "acq_chains": nch,
        },
        "real_time_factor": round(value * 1e6 / FS, 2),
    }
    if args.only:
        line["diagnostic_only_stage"] = args.only
    if not args.no_profile_events and stage_n[1] > 0:
        # the batch runs as interleaved chains (gsdr_acq split), so a step holds
        # stage_n / steps launches of each stage, each over B * steps / stage_n blocks
        corr_launch_s = stage_ms[1] / stage_n[1] / 1e3
        blocks_per_launch = B * args.steps / stage_n[1]
        # the nch chains' correlate launches run concurrently (one per stream, same
        # duration): the chip's correlate throughput is nch launches per launch time
        achieved = correlate_kernel_bytes_per_block() * blocks_per_launch * nch / corr_launch_s
        pmc = load_pmc_traffic()
        traffic = None
        if pmc and pmc.get("kernel") == "acq_correlate_kernel" and pmc.get("blocks"):
            # PMC HBM bytes of one launch over pmc["blocks"] blocks, per block x this launch's blocks
            traffic = pmc.get("hbm_bytes_per_launch") / pmc["blocks"] * blocks_per_launch
        line["roofline"] = {
            "bound": "hbm", "achieved": round(achieved / 1e9, 2), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK, 4), "traffic": traffic,
            "kernel": "acq_correlate_kernel", "avg_launch_us": round(corr_launch_s * 1e6, 2),
            "blocks_per_launch": blocks_per_launch, "concurrent_launches": nch,
            "algorithmic_bytes_per_launch": int(correlate_kernel_bytes_per_block() * blocks_per_launch),
        }
        line["stages_us_per_launch"] = {
            "acq_forward": round(stage_ms[0] / max(stage_n[0], 1) * 1e3, 2),
            "acq_correlate": round(stage_ms[1] / max(stage_n[1], 1) * 1e3, 2),
            "acq_reduce": round(stage_ms[2] / max(stage_n[2], 1) * 1e3, 2),
            "trk_loop_all_epochs": round(trk_ms / max(trk_launches, 1) * 1e3, 2),
            "trk_launch_covers_steps": K if args.trk_stream else 1,
            "acq_launches_per_step": round(stage_n[1] / args.steps, 2),
        }
    line["acq_roof_frac_whole_step"] = round(acq_bytes_per_block() * B / (ms_per_step / 1e3) / HBM_PEAK, 4)
    line["check"] = {"visible": len(vis), "acquired_block0": len(vis & det),
                     "median_prompt_over_early": round(prompt_ratio, 2), "trk_calls_per_channel": int(nrec.min()),
                     "trk_calls_per_channel_timed": trk_calls_timed,
                     "median_mean16_doppler_err_hz": None if dop_err is None else round(float(np.median(dop_err)), 2),
                     "channels_within_25hz": None if dop_err is None else int(np.sum(dop_err < 25.0))}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(iq, codes, sats)
    if rank == 0:
        print(json.dumps(line), flush=True)
    trk.close()
    for a in acqs:
        a.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
