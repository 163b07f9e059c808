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
the acquisition blocks of a step are split over two handles (--acq-chains 2), each
on its own stream.
Whole-job throughput = blocks * 4000 samples * ranks / max-over-ranks wall time.
Before the W warmup steps, untimed acquisition passes run back to back for at least
--min-warmup-ms (default 250): the chip ramps its clocks under sustained load, and the
timed K steps then measure the steady state a continuously running receiver sees
(profiles/r06w); --min-warmup-ms 0 measures from a cold chip.

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


def correlate_kernel_flops_per_block():
    """Nominal FP32 work of the dominant kernel per block (SURVEY §8(d) F_acq's P*D
    term): per (d, p) the code product, the N-point FFT, |.|^2 and the row
    reductions, 5 N log2 N + 11 N."""
    return P * D * (5 * N * math.log2(N) + 11 * N)


FP32_PEAK = 157.3e12   # MI355X FP32 vector (= f32 MFMA) peak, MI355X_MICROARCH.md


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


def rank_plan(world, rank, blocks_per_rank, channels):
    """The job's shard map (gsdr.shard): one stream of
    world * blocks_per_rank blocks per step; this rank's acquisition block span
    and its tracking channels (c % world)."""
    from gsdr import shard
    total = world * blocks_per_rank
    return {"total_blocks": total, "blocks": shard.block_range(total, world, rank),
            "channels": [int(c) for c in shard.channels_of(channels, world, rank)]}


# ---------------------------------------------------------------- C5 workload
C5_FS = 25000000
C5_N = 25000            # samples per 1 ms block at 25 Msps
C5_CHANNELS = 256       # BASELINE C5: 256 channels sharded across the node's GPUs
C5_SHARE = (12, 12, 8)  # one 32-channel share: GPS L1 C/A, Galileo E1, BeiDou B1I
C5_COUNTS = tuple(x * C5_CHANNELS // 32 for x in C5_SHARE)  # Channels_1C / _1B / _B1 .count: 96, 96, 64


def c5_channel_signal(c):
    """Signal (0 GPS, 1 Galileo, 2 BeiDou) and satellite slot of global channel c,
    numbered as GNSS-SDR numbers a .conf's channels: the Channels_1C.count GPS
    channels first, then Galileo, then BeiDou -- so the map c % world hands every
    GPU of an 8-GPU node the 12 + 12 + 8 share of SURVEY 8(d)."""
    c = int(c)
    if c < C5_COUNTS[0]:
        return 0, c % C5_SHARE[0]
    if c < C5_COUNTS[0] + C5_COUNTS[1]:
        return 1, (c - C5_COUNTS[0]) % C5_SHARE[1]
    return 2, (c - C5_COUNTS[0] - C5_COUNTS[1]) % C5_SHARE[2]


def c5_rank_plan(world, rank, blocks_per_rank, channels=C5_CHANNELS):
    """The C5 job's shard map (SURVEY 8e, weak scaling): one 25 Msps stream of
    world * blocks_per_rank 1 ms blocks per step; rank r acquires its block span
    (every 4 ms group: GPS L1 C/A grids on its even milliseconds, BeiDou B1I grids on
    the odd ones, one Galileo E1 4 ms grid) and tracks channels c % world of the 256
    over the whole span -- per-rank work stays constant as the world grows, and the
    channel -> GPU map replaces cuda_multicorrelator.cu:135-155's rand() % num_devices."""
    from gsdr import shard
    if blocks_per_rank % 4:
        raise ValueError("C5 blocks per rank must be a multiple of 4 (the Galileo 4 ms grid)")
    total = world * blocks_per_rank
    lo, hi = shard.block_range(total, world, rank)
    chans = [int(c) for c in shard.channels_of(channels, world, rank)]
    pools = {sig: [c for c in chans if c5_channel_signal(c)[0] == sig] for sig in (0, 1, 2)}
    return {"total_blocks": total, "blocks": (lo, hi), "channels": chans, "pools": pools,
            "acq": {"gps_blocks": list(range(lo, hi, 2)), "bds_blocks": list(range(lo + 1, hi, 2)),
                    "gal_groups": list(range(lo, hi, 4))}}


def host_cpu_info():
    """Threads the CPU baseline may use and what they are: the affinity set,
    capped by OMP_NUM_THREADS (the GPU box sets it to the job's CPU share; nproc
    there shows the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(aff, cap) if cap > 0 else aff
    model, cores = "unknown", None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") and model == "unknown":
                model = line.split(":", 1)[1].strip()
            if line.startswith("cpu cores") and cores is None:
                cores = int(line.split(":", 1)[1])
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": aff, "threads": threads, "cpu_model": model,
            "cores_per_socket": cores}


def cpu_baseline(iq, codes, sats, budget_s=12.0):
    """The C++ CPU restatement (oracle/cpu_baseline.cc) on this host's cores: per
    1 ms block the 32 PRN x 81 Doppler CFAR PCPS grid (own batched AVX2
    mixed-radix FFT -- no FFTW3f / pocketfft on the image -- std::thread over
    (Doppler bin, PRN group) tasks) plus one dll_pll_veml_tracking call per
    channel (fused AVX2 resampler + rotator correlator feeding the oracle's
    DLL/PLL restatement), on a bounded sample of blocks.  Also the per-core
    correlator rate (N=4000, K=3) for the fairness check against the reference's
    VOLK a_avx probe, 187 M channel-samples/s/core."""
    import ctypes
    from oracle import trk

    info = host_cpu_info()
    nt = info["threads"]
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libcpubase.so"))
    L.cpub_acq_create.restype = ctypes.c_void_p
    L.cpub_acq_create.argtypes = [ctypes.c_int] * 3 + [ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.cpub_acq_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    L.cpub_acq_destroy.argtypes = [ctypes.c_void_p]
    L.cpub_trk_calls.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_void_p]
    L.cpub_corr.argtypes = ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                             ctypes.c_int] + [ctypes.c_float] * 4 + [ctypes.c_int])
    from gsdr import synth
    codes_c = np.ascontiguousarray(codes, np.complex64)
    h = L.cpub_acq_create(N, D, P, float(FS), DMAX, DSTEP, codes_c.ctypes.data)
    nblk_data = len(iq) // N
    # the workload is periodic over its blocks (bench --trk-stream construction),
    # so channels read a doubled copy at their position modulo the period
    iq2 = np.ascontiguousarray(np.concatenate([iq, iq]), np.complex64)
    period = nblk_data * N
    chans, firsts = [], []
    for s in sats:
        o = trk.Channel(trk_conf(1).view(trk.TRK_CONF_DTYPE))
        delay, dop = acq_result_for(s)
        firsts.append(o.start(synth.gps_ca_chips(s.prn), delay, dop, 0, 0))
        chans.append(o)
    handles = (ctypes.c_void_p * len(chans))(*[o._h for o in chans])
    recs = np.zeros(len(chans), trk.TRK_EPOCH_DTYPE)
    out = np.zeros((P, 5), np.float32)
    pos = np.array(firsts, np.int64)

    def one_block(b):
        L.cpub_acq_run(h, iq[(b % nblk_data) * N:].ctypes.data, nt, out.ctypes.data)
        rel = (pos % period).astype(np.uint64)
        absn = pos.astype(np.uint64)
        L.cpub_trk_calls(handles, len(chans), iq2.ctypes.data, rel.ctypes.data, absn.ctypes.data, nt, recs.ctypes.data)
        pos[:] += recs["consumed"].astype(np.int64)

    # warm-up (thread pool, first touch, clocks), then size the sample from one block
    tw = time.perf_counter()
    nw = 0
    while time.perf_counter() - tw < 1.0 or nw < 2:
        one_block(nw)
        nw += 1
    t0 = time.perf_counter()
    one_block(1)
    t1 = time.perf_counter() - t0
    nblk = int(max(2, min(4000, math.ceil(budget_s / max(t1, 1e-4)))))
    t0 = time.perf_counter()
    for b in range(2, nblk + 2):
        one_block(b)
    dt = time.perf_counter() - t0
    # thread scaling inside the job's CPU share (short samples): how far the
    # measured figure is from a whole socket
    scaling = {}
    for tt in sorted({1, max(1, nt // 4), max(1, nt // 2), nt}):
        nt_saved = nt
        nt = tt
        tb = time.perf_counter()
        nb = 0
        while time.perf_counter() - tb < 1.5 or nb < 2:
            one_block(nblk + 2 + nb)
            nb += 1
        scaling[tt] = round(nb * N / (time.perf_counter() - tb) / 1e6, 4)
        nt = nt_saved
    detected = int(np.sum(out[:, 4] > 0))
    L.cpub_acq_destroy(h)
    # per-core correlator rate (1 thread, N = 4000, K = 3, L = 1023)
    code = synth.gps_ca_chips(1).astype(np.float32)
    shifts = np.array([-0.5, 0.0, 0.5], np.float32)
    o6 = np.zeros(6, np.float32)
    sig = np.ascontiguousarray(iq[:N], np.complex64)
    reps = 2000
    tc = time.perf_counter()
    for _ in range(reps):
        L.cpub_corr(o6.ctypes.data, sig.ctypes.data, code.ctypes.data, 1023, shifts.ctypes.data, 3, 0.3, 0.01, 0.1,
                    float(np.float32(1.023e6 / FS)), N)
    corr_rate = reps * N / (time.perf_counter() - tc) / 1e6
    value = nblk * N / dt / 1e6
    socket_cores = info.get("cores_per_socket") or nt
    # whole-socket estimate from the measured scaling curve (Amdahl's law fitted to
    # thread_scaling_msps: speedup(n) = 1 / (s + (1 - s) / n), s the median of the
    # per-point serial fractions), not a linear extrapolation
    r1 = scaling.get(1)
    fits = [((n / (r / r1)) - 1.0) / (n - 1.0) for n, r in scaling.items() if n > 1 and r1 and r > 0]
    serial = float(np.clip(np.median(fits), 0.0, 1.0)) if fits else 0.0
    socket_est = r1 / (serial + (1.0 - serial) / socket_cores) if r1 else value * socket_cores / nt
    return {"value": round(value, 4), "unit": "Msamples/s", "cores": nt, "kind": "port",
            "thread_scaling_msps": scaling,
            "full_socket_estimate": {"value": round(socket_est, 3), "cores": socket_cores,
                                     "serial_fraction": round(serial, 4),
                                     "linear_upper_bound": round(value * socket_cores / nt, 3),
                                     "basis": "Amdahl's law fitted to thread_scaling_msps (the job's CPU share is %d "
                                              "threads; the box's OMP/MAX_JOBS limit), evaluated at the socket's "
                                              "cores; an estimate, not a measurement" % nt},
            "sample": "%d blocks of 1 ms (4000 samples) in %.1f s: 32 PRN x 81 Doppler CFAR PCPS per block "
                      "(oracle/cpu_baseline.cc: own 8-lane AVX2 mixed-radix FFT, no FFTW3f/pocketfft on the image) "
                      "+ one dll_pll_veml_tracking call for each of 8 channels (fused AVX2 correlator + DLL/PLL "
                      "restatement), std::thread x %d" % (nblk, dt, nt),
            "host": info, "stats_checked_prns": detected,
            "per_core_correlator_Mchsps": round(corr_rate, 1),
            "fairness": "per-core correlator %.0f M ch-samples/s (N=4000, K=3) vs the reference VOLK a_avx probe "
                        "187 (BASELINE.md §2): %.2fx" % (corr_rate, corr_rate / 187.0)}


def achievable_hbm_gbps(torch, dev, mib=1024):
    """Achievable HBM bandwidth on this box ('also measure achievable BW
    with a copy kernel'): device-to-device copy of a `mib` MiB buffer, read + write
    bytes over the HIP-event time of the copy (median of 5)."""
    n = mib * (1 << 20) // 4
    a = torch.empty(n, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    a.fill_(1.0)
    b.copy_(a)
    ts = []
    for _ in range(5):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3)
    del a, b
    return 2.0 * n * 4 / sorted(ts)[2] / 1e9


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
                d["file"] = "profiles/" + f
                best = d
            except Exception:
                pass
    return best


def run_c5(args):
    """bench.py --workload c5: one step = a 25 Msps stream span of world x B 1 ms
    blocks; rank r runs the acquisition of its block span (c5_rank_plan: GPS L1 C/A
    and BeiDou B1I 32 PRN x 80 Doppler grids, N = 25000, on alternate milliseconds,
    one Galileo E1 36 PRN x 40 Doppler 4 ms grid, N = 100000, per 4 ms group; the
    reference's ceil(2 doppler_max / doppler_step) bins) and
    tracks its channels of the 256 (three signal pools, device-resident
    dll_pll_veml_tracking).  Tracking (default, as C2's --trk-stream) follows one
    continuous stream: the span is periodic (B = 100 ms: Galileo's 100 ms secondary
    code, carriers on whole cycles per span) and repeated end to end, one launch per
    pool covering all timed steps, so every channel is in steady state and even the
    4 ms Galileo channels make tens of calls per timed region; --trk-replay re-tracks
    the span from saved start states every step (B = 8 ms).  Inputs resident in HBM;
    value = world x B x 25000 samples per step / max-over-ranks time (weak scaling).
    Also reported: per-pool and acquisition-alone rates, the roofline of both stages,
    and the H2D ingest time of the rank's stream span (pinned host memory), which is
    never part of value."""
    import torch
    import gsdr
    from gsdr import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    local = rank_device(torch, local)
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if shared_device_rehearsal():
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    stream = not args.trk_replay
    B = args.blocks if args.blocks % 4 == 0 and args.blocks != 64 else (100 if stream else 8)
    W, K = args.warmup, args.steps
    plan = c5_rank_plan(world, rank, B)
    total = plan["total_blocks"]
    lo, hi = plan["blocks"]
    fs, n = C5_FS, C5_N
    # the stream: 12 GPS + 12 Galileo + 8 BeiDou satellites at 45 dB-Hz
    rng = np.random.default_rng(500)
    gps = synth.random_constellation(12, seed_offset=500, cn0_dbhz=45.0, prns=list(range(1, 13)), max_doppler=4000.0)
    gal = [synth.GalileoSatellite(p, float(rng.uniform(-4000, 4000)), float(rng.uniform(0, 4092)), 45.0,
                                  float(rng.uniform(0, 6.28))) for p in range(1, 13)]
    # BeiDou within +-1 kHz: the repeated span below carries no code Doppler (a code that
    # drifts with the carrier would jump at every repetition), and the carrier-aided B1I
    # DLL (1 Hz) follows the resulting code-rate mismatch only at low Doppler (beyond
    # ~2 kHz the channels lose 10 dB of CN0 and bias their Doppler, oracle and GPU alike)
    bds = [synth.Satellite(p, float(rng.uniform(-1000, 1000)) if stream else float(rng.uniform(-4000, 4000)),
                           float(rng.uniform(0, 2046)), 45.0, float(rng.uniform(0, 6.28)))
           for p in (6, 7, 8, 9, 10, 11, 12, 13)]
    if stream:
        # a whole number of carrier cycles per span: the span repeated end to end is a
        # continuous signal (no code Doppler; codes, secondary codes and data bits
        # are periodic in whole milliseconds of the span)
        span = total * n / fs
        for s in gps + gal + bds:
            s.doppler_hz = round(s.doppler_hz * span) / span
        ns = total * n
    else:
        ns = total * n + 4 * n  # + one Galileo code period of slack for the last calls
    iq = (synth.gps_l1_iq(fs, ns, gps, seed_offset=500, noise=False, dtype=np.complex128) +
          synth.gal_e1_iq(fs, ns, gal, seed_offset=500, noise=False, dtype=np.complex128) +
          synth.bds_b1i_iq(fs, ns, bds, seed_offset=500, noise=True, dtype=np.complex128,
                           code_doppler=not stream)).astype(np.complex64)
    iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    base = iq_dev.data_ptr()
    if stream:
        iq_long = iq_dev.repeat(W + K + 1)  # warmup + timed steps end to end, + one span of slack
        tbase, t_items = iq_long.data_ptr(), (W + K + 1) * ns
    else:
        iq_long, tbase, t_items = iq_dev, base, ns
    # acquisition handles of this rank's span
    acq_specs = (
        ("gps", n, 32, 10000, 250, 1, lambda: np.stack([synth.gps_ca_sampled(p, fs) for p in range(1, 33)]),
         plan["acq"]["gps_blocks"], 2),
        ("bds", n, 32, 10000, 250, 1, lambda: np.stack([synth.bds_b1i_sampled(p, fs)[:n] for p in range(1, 33)]),
         plan["acq"]["bds_blocks"], 2),
        ("gal", 4 * n, 36, 5000, 250, 4,
         lambda: np.stack([synth.gal_e1_sampled(p, fs, pilot=True)[:4 * n] for p in range(1, 37)]),
         plan["acq"]["gal_groups"], 4))
    acqs = []
    for name, N5, P5, dmax, dstep, ms, codes, blocks, stride_ms in acq_specs:
        if not blocks:
            continue
        a = gsdr.Acquisition(fs, N5, dmax, dstep, pfa=0.01, max_prns=P5, max_blocks=len(blocks), sampled_ms=ms,
                             ms_per_code=ms, chip_rate=2046000.0 if name == "bds" else 1023000.0, device=local)
        a.set_local_codes(codes(), np.arange(1, P5 + 1))
        res = torch.zeros(len(blocks) * P5 * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        acqs.append((name, a, blocks[0], len(blocks), stride_ms * n, res, P5, N5))
    # tracking pools: channel c tracks satellite slot i of its signal
    sats_of = (gps, gal, bds)
    pools = []
    for sig, chans in plan["pools"].items():
        if not chans:
            continue
        sigc = (gsdr.SIGNAL_GPS_1C, gsdr.SIGNAL_GAL_1B, gsdr.SIGNAL_BDS_B1)[sig]
        c = gsdr.trk_conf_default()
        c["fs_in"] = fs
        c["signal"] = sigc
        c["max_channels"] = len(chans)
        c["pll_bw_hz"], c["dll_bw_hz"] = (40.0, 4.0) if sig == 0 else (15.0, 1.0)
        if sig == 1:
            c["track_pilot"] = 1
        t = gsdr.Tracking(c, device=local)
        chip, per = ((1.023e6, n), (1.023e6, 4 * n), (2.046e6, n))[sig]
        truth = []
        for i, gc in enumerate(chans):
            s = sats_of[sig][c5_channel_signal(gc)[1]]
            truth.append(s.doppler_hz)
            tau = s.code_delay_chips / (chip * (1 + s.doppler_hz / 1.57542e9)) * fs
            # the acquisition's Doppler: the 250 Hz grid for GPS (40 Hz PLL); Galileo and
            # BeiDou (15 Hz PLLs) start from a make_two_steps refinement on a 25 Hz narrow grid
            grid = 250.0 if sig == 0 else 25.0
            dop = grid * round(s.doppler_hz / grid)
            if sig == 0:
                t.start(i, s.prn, synth.gps_ca_chips(s.prn), float(round(tau) % per), dop, 0, 0)
            elif sig == 1:
                t.start(i, s.prn, synth.gal_e1_sinboc11(s.prn, pilot=True), float(round(tau) % per), dop, 0, 0,
                        data_code=synth.gal_e1_sinboc11(s.prn))
            else:
                t.start(i, s.prn, synth.bds_b1i_chips(s.prn), float(round(tau) % per), dop, 0, 0)
        t.save_state(0)
        per_step = total * n // per  # general_work calls per channel per step
        epochs = (max(W, K) * per_step) if stream else per_step + 1
        out = torch.zeros(len(chans) * epochs * gsdr.TRK_EPOCH_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(len(chans), dtype=torch.int32, device=dev)
        pools.append(dict(sig=sig, t=t, per=per, per_step=per_step, epochs=epochs, out=out, cnt=cnt,
                          nch=len(chans), truth=np.array(truth)))

    def trk_launch(nsteps):
        # stream mode: one launch per pool for nsteps spans, continuing the stream
        for pl in pools:
            pl["t"].run_device(tbase, 0, t_items, nsteps * pl["per_step"], pl["out"].data_ptr(), pl["cnt"].data_ptr())

    step_no = [0]

    def acq_step(span=0):
        # stream mode: step k acquires span k of the continuous stream (new HBM
        # addresses every step, as the C2 line; not the same span re-read from L2)
        for name, a, b0, nb, stride, res, P5, N5 in acqs:
            a.run_device(tbase + (span * ns + b0 * n) * 8, nb, stride, span * ns + b0 * n, res.data_ptr())

    def step():
        if not stream:
            for pl in pools:
                pl["t"].restore_state(0)
                pl["t"].run_device(base, 0, ns, pl["epochs"], pl["out"].data_ptr(), pl["cnt"].data_ptr())
        acq_step(step_no[0] % (W + K + 1) if stream else 0)
        step_no[0] += 1

    prewarm_passes = clock_warmup(lambda k: acq_step(k % (W + K + 1) if stream else 0), args.min_warmup_ms,
                                  lambda: torch.cuda.synchronize(dev))
    if stream:
        trk_launch(W)
    for _ in range(W):
        step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if stream:
        trk_launch(K)
    for _ in range(K):
        step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_local = elapsed
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if shared_device_rehearsal() else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # sanity on the timed region's outputs: acquisitions of the visible satellites,
    # tracking records per channel, carrier Doppler of the last 16 calls vs the truth
    det = {}
    for name, a, b0, nb, stride, res, P5, N5 in acqs:
        r = res.cpu().numpy().view(gsdr.ACQ_RESULT_DTYPE).reshape(nb, P5)
        det[name] = sorted({int(x["prn"]) for x in r[0] if x["positive"]})
    names = ("gps", "gal", "bds")
    calls, conv = {}, {}
    for pl in pools:
        cnt = pl["cnt"].cpu().numpy()
        calls[names[pl["sig"]]] = int(cnt.min())
        recs = pl["out"].cpu().numpy().view(gsdr.TRK_EPOCH_DTYPE).reshape(pl["nch"], pl["epochs"])
        err = [abs(float(np.mean(recs[i][max(cnt[i] - 16, 0):cnt[i]]["carrier_doppler_hz"])) - pl["truth"][i])
               for i in range(pl["nch"]) if cnt[i] > 0]
        conv[names[pl["sig"]]] = {"median_mean16_doppler_err_hz": round(float(np.median(err)), 2) if err else None,
                                  "channels_within_25hz": int(np.sum(np.array(err) < 25.0)), "channels": pl["nch"]}
    flops = 0.0
    for name, a, b0, nb, stride, res, P5, N5 in acqs:
        Dn = a.num_doppler_bins
        flops += nb * (Dn * (5 * N5 * math.log2(N5) + 6 * N5) + P5 * Dn * (5 * N5 * math.log2(N5) + 11 * N5))
    samples = world * K * B * n
    value = samples / elapsed / 1e6

    def timed_part(fn):
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t1

    # components after the timed region: acquisition alone over K steps, each pool alone
    # over K spans (from its saved start state), the H2D ingest of the rank's span
    comp = {}
    ta = timed_part(lambda: [acq_step(k % (W + K + 1) if stream else 0) for k in range(K)])
    comp["acq_only_msps"] = round(B * n * K / ta / 1e6, 2)
    trk_bytes, trk_time = 0.0, 0.0
    for pl in pools:
        pl["t"].restore_state(0)
        if stream:
            tp = timed_part(lambda: pl["t"].run_device(tbase, 0, t_items, K * pl["per_step"], pl["out"].data_ptr(),
                                                       pl["cnt"].data_ptr()))
            span_items = K * total * n
        else:
            tp = timed_part(lambda: [(pl["t"].restore_state(0),
                                      pl["t"].run_device(base, 0, ns, pl["epochs"], pl["out"].data_ptr(),
                                                         pl["cnt"].data_ptr())) for _ in range(K)])
            span_items = K * total * n
        ncalls = int(pl["cnt"].cpu().numpy().sum())
        # algorithmic HBM bytes of a call: its IQ window (8 B per sample) + the record
        b = ncalls * (8.0 * pl["per"] + gsdr.TRK_EPOCH_DTYPE.itemsize)
        trk_bytes += b
        trk_time += tp
        comp["trk_%s_msps" % names[pl["sig"]]] = round(span_items / tp / 1e6, 2)
        comp["trk_%s_channels" % names[pl["sig"]]] = pl["nch"]
        comp["trk_%s_gbps" % names[pl["sig"]]] = round(b / tp / 1e9, 2)
    host = torch.from_numpy(iq.view(np.float32)).pin_memory()
    scratch = torch.empty_like(iq_dev)
    scratch.copy_(host, non_blocking=True)  # first touch
    th = timed_part(lambda: [scratch.copy_(host, non_blocking=True) for _ in range(4)]) / 4
    del scratch, host
    comp["note"] = ("each stage alone after the timed region over the same K spans; trk_<pool>_msps = the stream's IQ "
                    "rate through that pool (every channel processes every sample)")
    # where each rank's step goes: its own step time, the share of it
    # its acquisition grids alone take, and its pools' alone times -- gathered after the
    # timed region (the only collective besides the barriers and the max-over-ranks)
    mine = {"rank": rank, "step_ms": round(elapsed_local / K * 1e3, 4), "acq_only_ms_per_step": round(ta / K * 1e3, 4),
            "acq_fraction_of_step": round(ta / elapsed_local, 4), "trk_alone_ms_per_step": round(trk_time / K * 1e3, 4),
            "acq_blocks": [int(lo), int(hi)], "channels": len(plan["channels"])}
    if dist is not None:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
    else:
        gathered = [mine]
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded 25 Msps IQ: 12 GPS L1 C/A + 12 Galileo E1 + 8 BeiDou B1I at 45 dB-Hz + AWGN; "
                "one stream per job)",
        "config": {
            "workload": "C5: hybrid GPS L1 C/A + Galileo E1 + BeiDou B1I, 25 Msps, %d channels sharded c %% world "
                        "(12/12/8 per 32-channel share); per 4 ms of the rank's span 2 GPS + 2 BeiDou 32 PRN x 80 "
                        "Doppler grids (N 25000) and 1 Galileo 36 PRN x 40 Doppler grid (N 100000)" % C5_CHANNELS,
            "blocks_per_step": total, "blocks_per_rank": B, "fs_sps": fs,
            "parallelism": "one stream of %d ms per step: acquisition blocks [%d,%d) and %d channels (GPS %d, "
                           "Galileo %d, BeiDou %d) on rank %d of %d, no data-path collective"
                           % (total, lo, hi, len(plan["channels"]), len(plan["pools"][0]), len(plan["pools"][1]),
                              len(plan["pools"][2]), rank, world),
            "tracking": ("one continuous stream (periodic %d ms span repeated end to end), one launch per pool per "
                         "timed region" % total if stream else
                         "each step re-tracks the span from the channels' saved start states (one launch per pool)")},
        "real_time_factor": round(value * 1e6 / fs, 2),
        "roofline": {"bound": "valu", "achieved": round(flops * K / elapsed / 1e12, 2), "peak": FP32_PEAK / 1e12,
                     "unit": "TFLOP/s", "frac": round(flops * K / elapsed / FP32_PEAK, 4), "traffic": None,
                     "note": "nominal FFT flops of the rank's acquisition grids over the whole step (tracking and "
                             "acquisition share the GPU)",
                     "acquisition_alone": {"achieved": round(flops * K / ta / 1e12, 2), "unit": "TFLOP/s",
                                           "frac": round(flops * K / ta / FP32_PEAK, 4)},
                     "tracking_alone": {"bound": "hbm", "achieved": round(trk_bytes / trk_time / 1e9, 2),
                                        "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                                        "frac": round(trk_bytes / trk_time / HBM_PEAK, 5),
                                        "note": "each pool's calls x (8 B x vector_length + one record) over the "
                                                "pools' summed alone time: a serial per-channel loop, latency-bound"}},
        "components": comp,
        "per_rank": gathered,
        "h2d_ingest": {"bytes_per_step": int(ns * 8), "ms_per_step": round(th * 1e3, 3),
                       "gbps": round(ns * 8 / th / 1e9, 2), "frac_of_step": round(th / (elapsed / K), 4),
                       "note": "pinned host -> HBM copy of the rank's stream span per step (every rank ingests the "
                               "whole stream); not part of value"},
        "check": {"acquired_block0": det, "trk_calls_min_per_pool": calls, "tracking_convergence": conv,
                  "notes": ("stream mode: each step acquires its own span of the continuous stream; BeiDou Dopplers "
                            "drawn within +-1 kHz (the repeated span carries no code Doppler), so the BeiDou "
                            "convergence is not comparable with full-Doppler runs" if stream else
                            "replay mode: the same span every step, full +-4 kHz Dopplers")},
        "cpu_baseline": None,
        "prewarm": {"min_ms": args.min_warmup_ms, "acq_passes": prewarm_passes,
                    "note": "untimed acquisition passes before the W warmup steps (GPU clock ramp)"},
    }
    if shared_device_rehearsal() and world > 1:
        line["rehearsal"] = ("%d ranks sharing %d device(s) over gloo (GSDR_BENCH_SHARED_DEVICE): the multi-rank "
                             "path on real engines, not a scaling number" % (world, torch.cuda.device_count()))
    if rank == 0:
        print(json.dumps(line), flush=True)
    for pl in pools:
        pl["t"].close()
    for _, a, *_ in acqs:
        a.close()
    if dist is not None:
        dist.destroy_process_group()


def clock_warmup(acq_pass, ms, sync):
    """Untimed acquisition passes for at least `ms` ms, issued back to back before the W
    warmup steps: the MI355X ramps its clocks under sustained load and drops them in idle
    gaps, so with the driver's 5 warmup steps (6 ms at C2) the timed steps ran on a chip
    still ramping -- the same correlate kernel 1081-1084 us per launch after 5 warmup
    steps against 974-984 us after 200 (profiles/r06v).  The timed region is unchanged:
    exactly K full steps between the barriers.  Returns the passes run."""
    if ms <= 0:
        return 0
    # a short synchronised burst sizes one pass, then the rest go back to back with no
    # host synchronisation (an idle gap between passes lets the clocks drop again)
    t = time.perf_counter()
    n = 0
    for _ in range(4):
        acq_pass(n)
        n += 1
    sync()
    per = max((time.perf_counter() - t) / 4, 1e-5)
    rest = int(min(max(ms / 1e3 - 4 * per, 0.0) / per, 100000))
    for _ in range(rest):
        acq_pass(n)
        n += 1
    return n


# GSDR_BENCH_SHARED_DEVICE=1: a multi-rank rehearsal on a box with fewer GPUs than ranks --
# rank r uses device LOCAL_RANK % device_count() and the rank collectives run over gloo
# (RCCL refuses two ranks on one device).  Every rank runs the real engines on its share
# of the stream; the line is marked "rehearsal" and is never a scaling number.
def shared_device_rehearsal():
    return os.environ.get("GSDR_BENCH_SHARED_DEVICE", "0") == "1"


def rank_device(torch, local):
    if shared_device_rehearsal():
        return local % max(1, torch.cuda.device_count())
    return local


class DeviceBackend:
    """The device side of the C2 bench: torch's HIP device (HBM buffers, stream
    synchronisation, events), the gsdr engine and the rank collective's backend
    (RCCL: "nccl").  tests/test_shard_gloo.py substitutes a CPU stand-in (gloo,
    stubbed engine calls) to rehearse the multi-rank control flow -- process-group
    init, the barriers, the max-over-ranks timing, each rank's block span and
    channel set -- without a GPU (the replaced device split:
    cuda_multicorrelator.cu:135-155)."""

    dist_backend = "nccl"

    def __init__(self, local):
        import torch
        import gsdr
        self.torch, self.gsdr = torch, gsdr
        local = rank_device(torch, local)
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        if shared_device_rehearsal():
            self.dist_backend = "gloo"

    def dist_kwargs(self):
        return {} if self.dist_backend == "gloo" else {"device_id": self.dev}

    def synchronize(self):
        self.torch.cuda.synchronize(self.dev)

    def event(self):
        return self.torch.cuda.Event(enable_timing=True)


def main(argv=None, backend=DeviceBackend):
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
    ap.add_argument("--acq-sizes", default="",
                    help="comma list of the chains' block counts (sum = --blocks), overriding --acq-chains: unequal "
                         "chains drift out of step, so one chain's forward / reduce / argmax launches overlap the "
                         "other's correlate instead of coinciding with it")
    ap.add_argument("--min-warmup-ms", type=float, default=250.0,
                    help="before the W warmup steps, untimed acquisition passes for at least this long (GPU clock "
                         "ramp; 0: none) -- the timed region is still exactly K steps")
    ap.add_argument("--acq-stagger", type=int, default=0,
                    help="two chains: move this many blocks from one chain to the other on alternate steps "
                         "(sizes B/2 + s, B/2 - s, then B/2 - s, B/2 + s), so the chains' forward / reduce / argmax "
                         "launches fall inside the other chain's correlate instead of coinciding; every step still "
                         "acquires its B blocks")
    ap.add_argument("--trk-stream", action="store_true",
                    help="(default) tracking follows one continuous stream: the batch repeated end to end (Dopplers on "
                         "whole cycles per batch, so the repetition is a continuous signal), one tracking launch "
                         "covering all timed steps -- every channel converges as a receiver's would")
    ap.add_argument("--trk-replay", action="store_true",
                    help="re-track the same 64 ms from a saved start state every step (the pull-in transient each "
                         "time; one tracking launch per step)")
    ap.add_argument("--only", choices=["acq", "trk"], default=None,
                    help="diagnostic: run only one of the two stages (the line is then not the metric)")
    ap.add_argument("--workload", choices=["c2", "c5"], default="c2",
                    help="c2 (default, the metric's configuration) or c5: the 25 Msps hybrid GPS/Galileo/BeiDou "
                         "job, 256 channels sharded c %% world, acquisition block spans per rank")
    args = ap.parse_args(argv)
    args.trk_stream = not args.trk_replay
    if args.workload == "c5":
        return run_c5(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    be = backend(local)
    torch, gsdr, dev = be.torch, be.gsdr, be.dev
    if getattr(dev, "type", None) == "cuda":
        local = dev.index  # the engines' device (GSDR_BENCH_SHARED_DEVICE maps ranks onto fewer GPUs)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(be.dist_backend, **be.dist_kwargs())
    B = args.blocks
    W, K = args.warmup, args.steps
    # One stream for the whole job: every rank ingests the full
    # stream of world*B blocks per step; rank r acquires its block span
    # (gsdr.shard.block_range) and tracks channels c % world == r over the whole
    # span (gsdr.shard.channels_of).  No data-path collective.
    plan = rank_plan(world, rank, B, CHANNELS)
    total = plan["total_blocks"]
    lo, hi = plan["blocks"]
    my_ch = plan["channels"]
    sats, iq, codes = make_workload(total, 0, periodic=True)
    iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
    res_dev = torch.zeros(B * P * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    nloc = max(1, len(my_ch))
    if args.trk_stream:
        # the tracking stream: warmup + timed steps end to end
        iq_long = iq_dev.repeat(W + K + 1)  # + one step of slack for the last calls
        trk_epochs = max(W, K) * total
    else:
        iq_long = iq_dev
        trk_epochs = total
    trk_out = torch.zeros(nloc * trk_epochs * gsdr.TRK_EPOCH_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    trk_n = torch.zeros(nloc, dtype=torch.int32, device=dev)

    if args.acq_sizes:
        sizes = [int(v) for v in args.acq_sizes.split(",")]
        assert sum(sizes) == B and min(sizes) > 0, "--acq-sizes must sum to --blocks"
    else:
        nch0 = max(1, args.acq_chains)
        assert B % nch0 == 0, "--blocks must be a multiple of --acq-chains"
        sizes = [B // nch0] * nch0
    nch = len(sizes)
    stagger = args.acq_stagger if (nch == 2 and not args.acq_sizes) else 0
    assert 0 <= stagger < sizes[0], "--acq-stagger must be below the chain size"
    # per-step chain sizes: alternate steps swap which chain takes the extra blocks
    step_sizes = ([sizes[0] + stagger, sizes[1] - stagger], [sizes[0] - stagger, sizes[1] + stagger]) if stagger \
        else (sizes, sizes)
    acqs = []
    for i in range(nch):
        a = gsdr.Acquisition(FS, N, DMAX, DSTEP, pfa=PFA, max_prns=P, max_blocks=sizes[i] + stagger, num_doppler_bins=D,
                             device=local)
        a.set_local_codes(codes, np.arange(1, P + 1))
        acqs.append(a)
    trk = gsdr.Tracking(trk_conf(nloc), device=local) if len(my_ch) else None
    from gsdr import synth
    for i, c in enumerate(my_ch):
        s = sats[c]
        delay, dop = acq_result_for(s)
        trk.start(i, s.prn, synth.gps_ca_chips(s.prn), delay, dop, 0, 0)
    # each handle launches on its own HIP stream (its own hardware queue).  The
    # tracking pool is a latency chain of one workgroup per channel that needs a
    # whole CU; --cu-partition gives it CUs of its own and the acquisition grid
    # the rest, so neither waits for the other's workgroups to drain.
    if args.cu_partition and trk is not None:
        trk_mask, acq_mask = gsdr.cu_partition(args.trk_cus or nloc)
        trk.set_cu_mask(trk_mask)
        for a in acqs:
            a.set_cu_mask(acq_mask)
    if trk is not None:
        trk.save_state(0)
    do_trk = args.only != "acq" and trk is not None

    def trk_stream_launch(nsteps):
        # one launch: nsteps * total general_work calls per channel, continuing the stream
        if do_trk and nsteps > 0:
            trk.run_device(iq_long.data_ptr(), 0, (W + K + 1) * total * N, nsteps * total, trk_out.data_ptr(),
                           trk_n.data_ptr())

    step_no = [0]

    def acq_pass(k):
        # with the continuous stream each step acquires its own span of it (new HBM
        # addresses every step, as a receiver's ingest would be; not the same 2 MB
        # re-read from L2 / MALL)
        span = k % (W + K + 1) if args.trk_stream else 0
        src = iq_long if args.trk_stream else iq_dev
        sz = step_sizes[k % 2]
        off = 0
        for i, a in enumerate(acqs):
            b0 = lo + off
            a.run_device(src.data_ptr() + (span * total + b0) * N * 8, sz[i], N, (span * total + b0) * N,
                         res_dev.data_ptr() + off * P * gsdr.ACQ_RESULT_DTYPE.itemsize)
            off += sz[i]

    def step():
        if do_trk and not args.trk_stream:
            trk.restore_state(0)
            trk.run_device(iq_dev.data_ptr(), 0, total * N, total, trk_out.data_ptr(), trk_n.data_ptr())
        if args.only != "trk":
            acq_pass(step_no[0])
        step_no[0] += 1

    prewarm_passes = clock_warmup(acq_pass, args.min_warmup_ms if args.only != "trk" else 0.0, be.synchronize)

    if args.trk_stream:
        trk_stream_launch(W)
    for _ in range(args.warmup):
        step()
    # The sanity check below reads the timed region's own outputs after it ends, so
    # the GPU goes from the warmup steps straight into the timed steps instead of
    # idling while the host inspects results (an idle gap lets the clocks drop).
    if not args.no_profile_events:
        for a in acqs:
            a.set_profiling(True)
            a.read_profile()
        if trk is not None:
            trk.set_profiling(True)
            trk.read_profile()
    if dist is not None:
        dist.barrier()
    be.synchronize()
    # common time base for the chains' stage intervals (their busy-time union)
    ref_ev = None if args.no_profile_events else be.event()
    if ref_ev is not None:
        ref_ev.record()
    t0 = time.perf_counter()
    if args.trk_stream:
        trk_stream_launch(K)
    for _ in range(args.steps):
        step()
    be.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if shared_device_rehearsal() else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    trk_calls_timed = int(trk_n.cpu().numpy().min()) if do_trk else 0
    # sanity, on the timed region's outputs: the visible satellites are acquired
    # (every step acquires the same blocks) and tracked with a strong prompt (the
    # continuous stream's last calls; with --trk-replay the last step's 64 ms)
    res = res_dev.cpu().numpy().view(gsdr.ACQ_RESULT_DTYPE).reshape(B, P)
    det = {int(r["prn"]) for r in res[0] if r["positive"]}
    vis = {s.prn for s in sats}
    prompt_ratio, dop_err, nrec = None, None, np.zeros(1, np.int64)
    if do_trk:
        ep_chk = K * total if args.trk_stream else total  # the timed launch's max_epochs (record layout)
        recs = trk_out.cpu().numpy().view(gsdr.TRK_EPOCH_DTYPE)[:nloc * ep_chk].reshape(nloc, ep_chk)
        nrec = trk_n.cpu().numpy()
        taps = np.stack([recs[i][nrec[i] - 1]["taps"][:6].view(np.complex64) for i in range(nloc)])
        prompt_ratio = float(np.median(np.abs(taps[:, 1]) / np.maximum(np.abs(taps[:, 0]), 1e-9)))
        # carrier Doppler averaged over the last 16 calls (one call's value carries
        # the PLL's per-epoch jitter at 40 Hz loop bandwidth)
        if nrec.min() > 0:
            dop_err = np.array([abs(np.mean(recs[i][max(nrec[i] - 16, 0):nrec[i]]["carrier_doppler_hz"]) -
                                    sats[c].doppler_hz) for i, c in enumerate(my_ch)])
    stage_ms, stage_n, stage_busy = (np.zeros(4), np.zeros(4, np.uint32), np.zeros(4))
    trk_ms, trk_launches = 0.0, 0
    corr_union_ms = None
    if not args.no_profile_events:
        # the correlate stage's busy time over all chains: the union of every
        # launch interval of every handle against one reference event
        iv = []
        for a in acqs:
            st, en = a.read_profile_intervals(ref_ev.cuda_event, 1)
            iv += list(zip(st.tolist(), en.tolist()))
        if iv:
            iv.sort()
            corr_union_ms, lo_t, hi_t = 0.0, iv[0][0], iv[0][1]
            for x0, x1 in iv[1:]:
                if x0 > hi_t:
                    corr_union_ms += hi_t - lo_t
                    lo_t, hi_t = x0, x1
                else:
                    hi_t = max(hi_t, x1)
            corr_union_ms += hi_t - lo_t
        for a in acqs:
            ms_a, n_a, busy_a = a.read_profile_ex()
            stage_ms = stage_ms + ms_a
            stage_n = stage_n + n_a
            stage_busy = stage_busy + busy_a
        if trk is not None:
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
        "data": "synthetic (seeded GPS L1 C/A IQ, 8 visible PRNs at 45 dB-Hz + AWGN; one stream per job)",
        "config": {
            "workload": "C2: GPS L1 C/A 4 Msps; per 1 ms block a 32 PRN x 81 Doppler (+-10 kHz, 250 Hz) CFAR PCPS "
                        "grid + closed-loop DLL/PLL tracking (3-tap E-P-L, dll_pll_veml_tracking) of 8 channels "
                        "over the same span",
            "blocks_per_step": B, "fs_sps": FS, "fft_size": N, "prns": P, "doppler_bins": D, "channels": CHANNELS,
            "taps": TAPS, "item_type": "gr_complex",
            "parallelism": "one stream of %d blocks per step: acquisition blocks [%d,%d) and channels %s on rank %d "
                           "of %d (gsdr.shard), no data-path collective" % (total, lo, hi, my_ch, rank, world),
            "tracking": ("one continuous stream, one launch per timed region" if args.trk_stream
                         else "the step's span re-tracked from a saved state, one launch per step"),
            "cu_partition": ({"tracking": args.trk_cus or nloc, "acquisition": 256 - (args.trk_cus or nloc)}
                             if args.cu_partition else None),
            "acq_chains": nch,
            "acq_chain_blocks": sizes,
            "acq_stagger": stagger,
            "acq_input": ("each step acquires its own span of the continuous stream (new HBM addresses)"
                          if args.trk_stream else "the same span every step"),
            # the carrier model and the forward spectra computed per block (include/gsdr.h
            # gsdr_acq_set_wipeoff / gsdr_acq_get_spectrum_reuse)
            "carrier": ["exact", "generic", "avx2"][acqs[0].wipe_mode],
            "forward_spectra_per_block": acqs[0].spectrum_reuse[0],
        },
        "real_time_factor": round(value * 1e6 / FS, 2),
        "prewarm": {"min_ms": args.min_warmup_ms, "acq_passes": prewarm_passes,
                    "note": "untimed acquisition passes before the W warmup steps (GPU clock ramp)"},
    }
    if args.only:
        line["diagnostic_only_stage"] = args.only
    if not args.no_profile_events and stage_n[1] > 0:
        # a step holds stage_n / steps correlate launches (one per chain), each over
        # B * steps / stage_n blocks.  The chains' launches run concurrently on
        # their streams and share the chip, so a launch's duration counts the time
        # it shares with the other chain; the kernel's wall time is the union of all
        # chains' launch intervals against one reference event
        # (gsdr_acq_read_profile_intervals)
        corr_launch_s = stage_ms[1] / stage_n[1] / 1e3
        blocks_per_launch = B * args.steps / stage_n[1]
        corr_busy_s = (corr_union_ms / 1e3 if corr_union_ms is not None
                       else (stage_busy[1] / 1e3 if nch == 1 else corr_launch_s * stage_n[1] / nch))
        blocks_timed = B * args.steps
        achieved = correlate_kernel_bytes_per_block() * blocks_timed / corr_busy_s
        pmc = load_pmc_traffic()
        traffic = None
        kc_pmc = (pmc or {}).get("kernels", {}).get("acq_correlate_kernel", {})
        if pmc and pmc.get("blocks") and kc_pmc.get("hbm_bytes_per_launch"):
            # PMC HBM bytes per block (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction) x this launch's blocks
            traffic = kc_pmc["hbm_bytes_per_launch"] / pmc["blocks"] * blocks_per_launch
        # The correlate kernel is not HBM bound: its spectra come from HBM once and
        # are re-served from L2 / the Infinity Cache to the 32 PRN workgroups (PMC
        # traffic below); its time is VALU issue (packed-f32 butterflies) plus the
        # LDS round trips and barriers between stages.  The roofline
        # is therefore the FP32 vector peak with the nominal FFT flops; the
        # logical-byte HBM figure and this box's achievable copy rate are kept alongside.
        flops = correlate_kernel_flops_per_block() * blocks_timed / corr_busy_s
        line["roofline"] = {
            "bound": "valu", "achieved": round(flops / 1e12, 2), "peak": FP32_PEAK / 1e12, "unit": "TFLOP/s",
            "frac": round(flops / FP32_PEAK, 4), "traffic": traffic,
            "traffic_source": (pmc or {}).get("file"),
            "kernel": "acq_correlate_pk_kernel", "avg_launch_us": round(corr_launch_s * 1e6, 2),
            "busy_us_per_step": round(corr_busy_s / args.steps * 1e6, 2),
            "busy_source": ("union of every chain's correlate launch intervals (one reference event)"
                            if corr_union_ms is not None else "per-handle busy time"),
            "blocks_per_launch": blocks_per_launch,
            "launch_overlap": round(corr_launch_s * stage_n[1] / corr_busy_s, 3),
            "nominal_flops_per_launch": int(correlate_kernel_flops_per_block() * blocks_per_launch),
            "hbm_logical": {"achieved": round(achieved / 1e9, 2), "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                            "achievable_copy": round(achievable_hbm_gbps(torch, dev), 1),
                            "frac": round(achieved / HBM_PEAK, 4),
                            "algorithmic_bytes_per_launch": int(correlate_kernel_bytes_per_block() * blocks_per_launch)},
        }
        if traffic:
            # the metric's "% HBM roofline" as measured: the PMC's HBM bytes of the
            # correlate grid over its busy time, against the 8 TB/s peak
            meas = traffic * stage_n[1] / corr_busy_s
            line["roofline"]["hbm_measured"] = {"achieved": round(meas / 1e9, 2), "peak": HBM_PEAK / 1e9,
                                                "unit": "GB/s", "frac": round(meas / HBM_PEAK, 4),
                                                "bytes_per_launch": round(traffic)}
        if pmc:
            kc = pmc.get("kernels", {}).get("acq_correlate_kernel", {}).get("counters", {})
            if kc.get("SQ_INSTS_VALU") and pmc.get("blocks"):
                line["roofline"]["pmc"] = {
                    "source": pmc.get("file"),
                    "valu_wave_instructions_per_block": round(kc["SQ_INSTS_VALU"] / pmc["blocks"]),
                    # bank-conflict cycles over all LDS-array cycles (SQ_LDS_IDX_ACTIVE,
                    # MI355X_MICROARCH.md LDS); older summaries lack that counter
                    "lds_bank_conflict_frac": (round(kc["SQ_LDS_BANK_CONFLICT"] / kc["SQ_LDS_IDX_ACTIVE"], 3)
                                               if kc.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in kc else None),
                    "hbm_bytes_per_block": round(pmc["hbm_bytes_per_launch"] / pmc["blocks"]) if pmc.get("hbm_bytes_per_launch") else None,
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
                     "median_prompt_over_early": None if prompt_ratio is None else round(prompt_ratio, 2),
                     "prompt_over_early_theory": round(1.0 / (1.0 - 0.25), 2),
                     "trk_calls_per_channel": int(nrec.min()),
                     "trk_calls_per_channel_timed": trk_calls_timed,
                     "median_mean16_doppler_err_hz": None if dop_err is None else round(float(np.median(dop_err)), 2),
                     "channels_within_25hz": None if dop_err is None else int(np.sum(dop_err < 25.0))}
    # Acquisition-only and tracking-only rates, each timed over K steps
    # after the headline's timed region with the same handles: the acquisition
    # chains without the tracking launch, and the tracking launch alone (restarted
    # from the saved start state, K steps of the continuous stream).
    if args.only is None and do_trk and args.trk_stream:
        if not args.no_profile_events:
            for a in acqs:
                a.set_profiling(False)
            trk.set_profiling(False)

        def timed_part(fn):
            be.synchronize()
            t = time.perf_counter()
            fn()
            be.synchronize()
            return time.perf_counter() - t

        def acq_only():
            for k in range(K):
                span = k if args.trk_stream else 0  # the timed region's spans (step())
                src = iq_long if args.trk_stream else iq_dev
                sz = step_sizes[k % 2]
                off = 0
                for i, a in enumerate(acqs):
                    b0 = lo + off
                    a.run_device(src.data_ptr() + (span * total + b0) * N * 8, sz[i], N, (span * total + b0) * N,
                                 res_dev.data_ptr() + off * P * gsdr.ACQ_RESULT_DTYPE.itemsize)
                    off += sz[i]

        def trk_only():
            trk.restore_state(0)
            trk.run_device(iq_long.data_ptr(), 0, (W + K + 1) * total * N, K * total, trk_out.data_ptr(),
                           trk_n.data_ptr())
        ta = timed_part(acq_only)
        tt = timed_part(trk_only)
        line["components"] = {
            "acq_only_msps": round(B * N * K / ta / 1e6, 2),
            "trk_only_msps": round(total * N * K / tt / 1e6, 2),
            "trk_only_channels": nloc,
            "note": "each over K steps after the timed region; trk_only = the stream's IQ rate through the tracking "
                    "pool (every channel processes every sample)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(iq, codes, sats)
    if shared_device_rehearsal() and world > 1:
        line["rehearsal"] = ("%d ranks sharing %d device(s) over gloo (GSDR_BENCH_SHARED_DEVICE): the multi-rank "
                             "path on real engines, not a scaling number" % (world, torch.cuda.device_count()))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if trk is not None:
        trk.close()
    for a in acqs:
        a.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
