#!/usr/bin/env python3
"""Throughput of the engine on BASELINE.json's other configurations (C3, C4, C5; C2
is bench.py's metric).  One JSON line per configuration and stage, inputs resident
in HBM before the timed region, HIP-synchronised wall time over `--reps`
repetitions after warm-up.  Msamples/s counts input-stream samples (every channel
and PRN of a stage works on the same stream), so real time = fs.

  C3  GPS L1 C/A 16 Msps: 12-channel 5-tap E-P-L multicorrelator epochs (gsdr_corr,
      shifts -0.5..0.5 chip), the 12-channel tracking loop, and the 32 PRN x 81
      Doppler acquisition grid (N = 16000)
  C4  Galileo E1 8 Msps (conf/gnss-sdr_galileo_E1_extended_correlator_byte.conf):
      8-channel VEML pilot tracking with 4-symbol extended integration, and the
      36 PRN x 80 Doppler acquisition with bit_transition_flag (N = 64000, four-step)
  C5  hybrid 25 Msps, one GPU's channel pool: 12 GPS + 12 Galileo + 8 BeiDou
      tracking channels (three handles on three streams)
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


WARM_MS = 250.0  # --warm-ms: the chip's clock ramp (bench.py clock_warmup)


def timed(fn, reps, warm, torch):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    if WARM_MS > 0:
        # untimed repetitions back to back for >= WARM_MS: the MI355X ramps its clocks under
        # sustained load (a 4-block C5 grid is < 1 ms; the timed reps alone ran on a cold chip)
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        per = max(time.perf_counter() - t, 1e-5)
        for _ in range(int(min(WARM_MS / 1e3 / per, 100000))):
            fn()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def emit(cfg, stage, fs, samples, sec, extra=None):
    d = {"config": cfg, "stage": stage, "fs_sps": fs, "msps": round(samples / sec / 1e6, 2),
         "real_time_factor": round(samples / sec / fs, 2), "ms_per_rep": round(sec * 1e3, 3)}
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


FP32_PEAK_TFLOPS = 157.3  # MI355X dense FP32 (vector), MI355X_MICROARCH.md


def acq_roofline(N, P, D, blocks, sec):
    """Nominal FFT flops of the PCPS grid: D forward transforms
    (5 N log2 N + 6 N: wipe-off product + FFT) and P*D correlate transforms
    (5 N log2 N + 11 N: product, FFT, |.|^2 and the row statistic) per block,
    against the FP32 peak -- the acquisition kernels are VALU-bound."""
    import math
    f = D * (5 * N * math.log2(N) + 6 * N) + P * D * (5 * N * math.log2(N) + 11 * N)
    tf = f * blocks / sec / 1e12
    return {"roofline": {"bound": "valu", "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tf / FP32_PEAK_TFLOPS, 4), "nominal_flops_per_block": round(f)}}


def trk_conf(gsdr, fs, sig, nch, **kw):
    c = gsdr.trk_conf_default()
    c["fs_in"] = fs
    c["signal"] = sig
    c["max_channels"] = nch
    for k, v in kw.items():
        c[k] = v
    return c


def main():
    global WARM_MS
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="C3,C4,C5")
    ap.add_argument("--acq-only", action="store_true", help="only the acquisition lines (A/B sweeps)")
    ap.add_argument("--warm-ms", type=float, default=WARM_MS,
                    help="untimed back-to-back repetitions before each timed line (GPU clock ramp; 0: none)")
    a = ap.parse_args()
    WARM_MS = a.warm_ms
    import torch
    import gsdr
    from gsdr import synth
    dev = torch.device("cuda", 0)
    todo = a.only.split(",")

    if "C3" in todo:
        fs, N, nch = 16000000, 16000, 12
        sats = synth.random_constellation(nch, seed_offset=3, prns=list(range(1, 13)))
        for s in sats:
            s.code_doppler = True
        ms = 100
        iq = synth.gps_l1_iq(fs, ms * N + N, sats, seed_offset=3)
        iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
        if not a.acq_only:
            # 5-tap multicorrelator epochs (one launch per epoch, 12 channel jobs)
            corr = gsdr.Correlator(nch, N + 64, max_taps=5)
            sh = np.array([-0.5, -0.25, 0.0, 0.25, 0.5], np.float32)
            for c, s in enumerate(sats):
                corr.set_local_code_and_taps(c, synth.gps_ca_chips(s.prn), sh)
            jl = []
            for e in range(ms):
                for c, s in enumerate(sats):
                    j = gsdr.CorrJob()
                    j.channel, j.n_samples, j.sample_offset = c, N, e * N
                    j.rem_carr_phase_rad = 0.1
                    j.carr_phase_step_rad = float(np.float32(2 * np.pi * s.doppler_hz / fs))
                    j.carr_phase_rate_step_rad = 0.0
                    j.rem_code_phase_chips = 0.3
                    j.code_phase_step_chips = float(np.float32(1.023e6 / fs))
                    j.code_phase_rate_step_chips = 0.0
                    jl.append(j)
            jarr = (gsdr.CorrJob * len(jl))(*jl)
            jbytes = bytes(jarr)
            jobs_dev = torch.frombuffer(bytearray(jbytes), dtype=torch.uint8).to(dev)
            out_dev = torch.zeros(ms * nch * 8 * 2, dtype=torch.float32, device=dev)
            sec = timed(lambda: corr.run_epochs(jobs_dev.data_ptr(), nch, ms, iq_dev.data_ptr(), len(iq), out_dev.data_ptr()),
                        a.reps, 3, torch)
            emit("C3", "multicorrelator 12 ch x 5 taps (epoch launches)", fs, ms * N, sec,
                 {"hbm_gbps_algorithmic": round(ms * nch * (8 * N + 8 * 5) / sec / 1e9, 1)})
            corr.close()
            # tracking loop, 12 channels
            trk = gsdr.Tracking(trk_conf(gsdr, fs, gsdr.SIGNAL_GPS_1C, nch, pll_bw_hz=40.0, dll_bw_hz=4.0))
            for c, s in enumerate(sats):
                tau = s.code_delay_chips / (1.023e6 * (1 + s.doppler_hz / 1.57542e9)) * fs
                trk.start(c, s.prn, synth.gps_ca_chips(s.prn), float(round(tau) % N), 250.0 * round(s.doppler_hz / 250.0), 0, 0)
            trk.save_state(0)
            out = torch.zeros(nch * ms * gsdr.TRK_EPOCH_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            nout = torch.zeros(nch, dtype=torch.int32, device=dev)

            def trk_step():
                trk.restore_state(0)
                trk.run_device(iq_dev.data_ptr(), 0, len(iq), ms - 1, out.data_ptr(), nout.data_ptr())
            sec = timed(trk_step, a.reps, 2, torch)
            emit("C3", "tracking loop 12 ch (3-tap dll_pll_veml_tracking)", fs, (ms - 1) * N, sec)
            trk.close()
        # acquisition grid
        B = 16
        acq = gsdr.Acquisition(fs, N, 10000, 250, pfa=0.01, max_prns=32, max_blocks=B, num_doppler_bins=81)
        acq.set_local_codes(np.stack([synth.gps_ca_sampled(p, fs) for p in range(1, 33)]), np.arange(1, 33))
        res = torch.zeros(B * 32 * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        sec = timed(lambda: acq.run_device(iq_dev.data_ptr(), B, N, 0, res.data_ptr()), a.reps, 3, torch)
        emit("C3", "acquisition 32 PRN x 81 Doppler, N=16000", fs, B * N, sec, acq_roofline(N, 32, 81, B, sec))
        acq.close()
        del iq_dev

    if "C4" in todo:
        fs, N, nch = 8000000, 32000, 8
        rng = np.random.default_rng(4)
        gsats = [synth.GalileoSatellite(p, float(rng.uniform(-4000, 4000)), float(rng.uniform(0, 4092)), 46.0,
                                        float(rng.uniform(0, 6.28))) for p in range(1, nch + 1)]
        calls = 60
        iq = synth.gal_e1_iq(fs, calls * N + 2 * N, gsats, seed_offset=4)
        iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
        if not a.acq_only:
            trk = gsdr.Tracking(trk_conf(gsdr, fs, gsdr.SIGNAL_GAL_1B, nch, track_pilot=1, pll_bw_hz=4.0, dll_bw_hz=0.5,
                                         pll_bw_narrow_hz=2.0, dll_bw_narrow_hz=0.25, extend_correlation_symbols=4,
                                         early_late_space_chips=0.15, very_early_late_space_chips=0.6,
                                         early_late_space_narrow_chips=0.06, very_early_late_space_narrow_chips=0.25))
            for c, s in enumerate(gsats):
                tau = s.code_delay_chips / (1.023e6 * (1 + s.doppler_hz / 1.57542e9)) * fs
                trk.start(c, s.prn, synth.gal_e1_sinboc11(s.prn, pilot=True), float(round(tau) % N),
                          125.0 * round(s.doppler_hz / 125.0), 0, 0, data_code=synth.gal_e1_sinboc11(s.prn))
            trk.save_state(0)
            out = torch.zeros(nch * calls * gsdr.TRK_EPOCH_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            nout = torch.zeros(nch, dtype=torch.int32, device=dev)

            def trk_step():
                trk.restore_state(0)
                trk.run_device(iq_dev.data_ptr(), 0, len(iq), calls, out.data_ptr(), nout.data_ptr())
            sec = timed(trk_step, a.reps, 2, torch)
            emit("C4", "tracking loop 8 ch Galileo E1 VEML pilot (+data prompt)", fs, calls * N, sec)
            trk.close()
        # acquisition, bit transition: 2 x 4 ms consumed, FFT 64000 (four-step), peak ratio
        B = 4
        acq = gsdr.Acquisition(fs, 2 * N, 5000, 125, pfa=0.0, max_prns=36, max_blocks=B, sampled_ms=4,
                               ms_per_code=4, bit_transition=True)
        codes = np.stack([np.resize(synth.gal_e1_sampled(p, fs, pilot=True), 2 * N) for p in range(1, 37)])
        acq.set_local_codes(codes, np.arange(1, 37))
        acq.set_threshold(2.5)
        res = torch.zeros(B * 36 * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        sec = timed(lambda: acq.run_device(iq_dev.data_ptr(), B, 2 * N, 0, res.data_ptr()), max(2, a.reps // 3), 1, torch)
        emit("C4", "acquisition 36 PRN x %d Doppler, bit transition, FFT %d" % (acq.num_doppler_bins, acq.fft_size),
             fs, B * 2 * N, sec, acq_roofline(2 * N, 36, acq.num_doppler_bins, B, sec))
        acq.close()
        # the same grid without bit transition: one 4 ms code period, FFT 32000
        acq = gsdr.Acquisition(fs, N, 5000, 125, pfa=0.0, max_prns=36, max_blocks=B, sampled_ms=4, ms_per_code=4)
        acq.set_local_codes(codes[:, :N], np.arange(1, 37))
        acq.set_threshold(2.5)
        sec = timed(lambda: acq.run_device(iq_dev.data_ptr(), B, N, 0, res.data_ptr()), max(2, a.reps // 3), 1, torch)
        emit("C4", "acquisition 36 PRN x %d Doppler, 4 ms, FFT %d" % (acq.num_doppler_bins, acq.fft_size),
             fs, B * N, sec, acq_roofline(N, 36, acq.num_doppler_bins, B, sec))
        acq.close()
        del iq_dev

    if "C5" in todo:
        fs = 25000000
        ms = 40
        gps = synth.random_constellation(12, seed_offset=5, prns=list(range(1, 13)))
        for s in gps:
            s.code_doppler = True
        iq = synth.gps_l1_iq(fs, ms * 25000 + 200000, gps, seed_offset=5)
        iq_dev = torch.from_numpy(iq.view(np.float32).copy()).to(dev)
        if not a.acq_only:
            rng = np.random.default_rng(5)
            pools = []
            conf_g = trk_conf(gsdr, fs, gsdr.SIGNAL_GPS_1C, 12, pll_bw_hz=40.0, dll_bw_hz=4.0)
            tg = gsdr.Tracking(conf_g)
            for c, s in enumerate(gps):
                tau = s.code_delay_chips / (1.023e6 * (1 + s.doppler_hz / 1.57542e9)) * fs
                tg.start(c, s.prn, synth.gps_ca_chips(s.prn), float(round(tau) % 25000), 250.0 * round(s.doppler_hz / 250.0), 0, 0)
            pools.append((tg, ms - 2))
            te = gsdr.Tracking(trk_conf(gsdr, fs, gsdr.SIGNAL_GAL_1B, 12, track_pilot=1, pll_bw_hz=15.0, dll_bw_hz=1.0))
            for c in range(12):
                te.start(c, c + 1, synth.gal_e1_sinboc11(c + 1, pilot=True), float(rng.integers(0, 100000)), 500.0, 0, 0,
                         data_code=synth.gal_e1_sinboc11(c + 1))
            pools.append((te, ms // 4 - 2))
            tb = gsdr.Tracking(trk_conf(gsdr, fs, gsdr.SIGNAL_BDS_B1, 8, pll_bw_hz=15.0, dll_bw_hz=1.0))
            for c in range(8):
                tb.start(c, 6 + c, synth.bds_b1i_chips(6 + c), float(rng.integers(0, 25000)), -750.0, 0, 0)
            pools.append((tb, ms - 2))
            bufs = []
            for t, n in pools:
                t.save_state(0)
                bufs.append((torch.zeros(t.max_channels * n * gsdr.TRK_EPOCH_DTYPE.itemsize, dtype=torch.uint8, device=dev),
                             torch.zeros(t.max_channels, dtype=torch.int32, device=dev)))

            def step():
                for (t, n), (o, no) in zip(pools, bufs):
                    t.restore_state(0)
                    t.run_device(iq_dev.data_ptr(), 0, len(iq), n, o.data_ptr(), no.data_ptr())
            sec = timed(step, a.reps, 2, torch)
            emit("C5", "tracking pool 12 GPS + 12 Galileo + 8 BeiDou (one GPU's share), three streams", fs,
                 (ms - 2) * 25000, sec)
            for t, _ in pools:
                t.close()
        # acquisition grids of one GPU's C5 share at 25 Msps: GPS L1 C/A and BeiDou B1I
        # (1 ms, N = 25000 = 5 x 5000 four-step), Galileo E1 (4 ms, N = 100000 = 25 x 4000)
        B = 4
        for name, N, P, dmax, dstep, codes in (
                ("GPS L1 C/A 32 PRN x %d Doppler, N=25000", 25000, 32, 10000, 250,
                 lambda: np.stack([synth.gps_ca_sampled(p, fs) for p in range(1, 33)])),
                ("BeiDou B1I 32 PRN x %d Doppler, N=25000", 25000, 32, 10000, 250,
                 lambda: np.stack([synth.bds_b1i_sampled(p, fs)[:25000] for p in range(1, 33)])),
                ("Galileo E1 36 PRN x %d Doppler, 4 ms, N=100000", 100000, 36, 5000, 250,
                 lambda: np.stack([synth.gal_e1_sampled(p, fs, pilot=True)[:100000] for p in range(1, 37)]))):
            ms_code = N // 25000
            acq = gsdr.Acquisition(fs, N, dmax, dstep, pfa=0.01, max_prns=P, max_blocks=B, sampled_ms=ms_code,
                                   ms_per_code=ms_code)
            acq.set_local_codes(codes(), np.arange(1, P + 1))
            res = torch.zeros(B * P * gsdr.ACQ_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            sec = timed(lambda: acq.run_device(iq_dev.data_ptr(), B, N, 0, res.data_ptr()), max(2, a.reps // 2), 1, torch)
            emit("C5", "acquisition " + name % acq.num_doppler_bins, fs, B * N, sec,
                 acq_roofline(N, P, acq.num_doppler_bins, B, sec))
            acq.close()


if __name__ == "__main__":
    main()
