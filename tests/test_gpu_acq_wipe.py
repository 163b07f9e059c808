"""The acquisition grid's carrier wipe-off models and the forward-spectrum reuse
(include/gsdr.h gsdr_acq_set_wipeoff / gsdr_acq_get_spectrum_reuse, acq_impl.h XMap),
through the C ABI.

GNSS-SDR computes each Doppler row's carrier with volk_gnsssdr_s32f_sincos_32fc
(pcps_acquisition.cc:233-246); which protokernel runs depends on the host: the
generic one (one fp32 phase accumulator, KERN/s32f_sincos_32fc.h:390-403) or, on an
AVX2 x86-64 host, a_avx2 (eight accumulators, Cephes polynomials, :448-627).  Their
accumulated phases drift from the exact carrier by different amounts, so the two
reference builds disagree by 4e-4 (C2) to 1e-2 (C4) of the peak.  The engine's
default is the exact carrier (and, for commensurate grids, every Doppler row as an
exact circular shift of q forward spectra); the bar:
  * GPU vs the fp64-carrier oracle: within 1e-4 (RTOL), cells equal or H3 near ties;
  * GPU vs each reference protokernel: within that protokernel's own distance from
    the exact carrier + 1e-4 of the peak;
  * GSDR_WIPE_GENERIC / GSDR_WIPE_AVX2: the protokernel replayed, parity with the
    oracle's replay at 1e-4 (the bar of tests/test_gpu_acq.py).
"""
import json
import os

import numpy as np
import pytest

import gsdr
from gsdr import synth
from oracle import pcps

pytestmark = pytest.mark.gpu

RTOL = 1e-4


def _log(line):
    print("parity acq_wipe", json.dumps(line))
    if os.environ.get("GSDR_PARITY_LOG"):
        with open(os.environ["GSDR_PARITY_LOG"], "a") as f:
            f.write(json.dumps(line) + "\n")


def _c2(seed=31, nprn=8):
    fs, N, dmax, dstep = 4000000, 4000, 10000, 250
    sats = synth.random_constellation(8, seed_offset=seed)
    x = synth.gps_l1_iq(fs, N, sats, seed_offset=seed)
    prns = np.array([s.prn for s in sats][:nprn])
    codes = np.stack([synth.gps_ca_sampled(int(p), fs, N) for p in prns])
    return dict(fs=fs, N=N, dmax=dmax, dstep=dstep, x=x, prns=prns, codes=codes, bt=False, spc=4, kw={})


def _c3(seed=33):
    fs, N, dmax, dstep = 16000000, 16000, 10000, 250
    sats = synth.random_constellation(6, seed_offset=seed)
    x = synth.gps_l1_iq(fs, N, sats, seed_offset=seed)
    prns = np.array([s.prn for s in sats][:4] + [31, 32])
    codes = np.stack([synth.gps_ca_sampled(int(p), fs, N) for p in prns])
    return dict(fs=fs, N=N, dmax=dmax, dstep=dstep, x=x, prns=prns, codes=codes, bt=False, spc=16, kw={})


def _c4bt(seed=64):
    fs, C, dmax, dstep = 8000000, 32000, 5000, 125
    rng = np.random.default_rng(seed)
    sats = [synth.GalileoSatellite(p, float(rng.uniform(-4500, 4500)), float(rng.uniform(0, 4092)), 45.0,
                                   float(rng.uniform(0, 6.28))) for p in (4, 19)]
    x = synth.gal_e1_iq(fs, 2 * C, sats, seed_offset=seed)
    prns = np.array([4, 7, 19, 30])
    codes = np.stack([np.resize(synth.gal_e1_sampled(int(p), fs), 2 * C) for p in prns])
    return dict(fs=fs, N=2 * C, dmax=dmax, dstep=dstep, x=x, prns=prns, codes=codes, bt=True, spc=8,
                kw=dict(bit_transition=True, sampled_ms=4, ms_per_code=4, samples_per_code=float(C)))


CONFIGS = {"C2": _c2, "C3": _c3, "C4bt": _c4bt}


def _acq(cfg, pfa, mode=None):
    acq = gsdr.Acquisition(cfg["fs"], cfg["N"], cfg["dmax"], cfg["dstep"], pfa=pfa, max_prns=len(cfg["prns"]),
                           **cfg["kw"])
    if mode is not None:
        acq.set_wipeoff(mode)
    acq.set_local_codes(cfg["codes"], cfg["prns"])
    if pfa == 0:
        acq.set_threshold(2.0)
    return acq


def _grids(cfg, D, mode):
    N = cfg["N"]
    wipe = pcps.doppler_wipeoffs(cfg["fs"], N, cfg["dmax"], cfg["dstep"], D, mode=mode)
    out = []
    for code in cfg["codes"]:
        cf = pcps.fft_code(code, N, N, bit_transition=cfg["bt"])
        out.append(pcps.magnitude_grid(cfg["x"], wipe, cf, bit_transition=cfg["bt"]))
    return out


def _stat(M, pfa, cfg):
    if pfa > 0:
        return pcps.max_to_input_power_statistic(M)
    N = cfg["N"]
    full = np.zeros((M.shape[0], N), np.float32)
    full[:, :M.shape[1]] = M
    return pcps.first_vs_second_peak_statistic(full, cfg["spc"], N)


def _check(r, M, pfa, cfg):
    """tests/test_gpu_acq.py's bar: cell equal (or an H3 near tie), values at RTOL."""
    ti, di, gmax, aux, stat = _stat(M, pfa, cfg)
    if (r["doppler_index"], r["code_phase"]) != (di, ti):
        assert abs(M[r["doppler_index"], r["code_phase"]] - gmax) <= RTOL * gmax, (r, ti, di)
        return False
    assert abs(r["peak"] - gmax) <= RTOL * gmax
    assert abs(r["test_statistic"] - stat) <= RTOL * stat
    assert abs((r["input_power"] if pfa > 0 else r["second_peak"]) - aux) <= RTOL * aux
    return True


def test_spectrum_reuse_factors():
    """q spectra per block and the shift p per class step (doppler_step N / fs = p / q)."""
    cases = [((4000000, 4000, 10000, 250, {}), (4, 1)),                 # C2: 250 Hz of 1 kHz bins
             ((8000000, 64000, 5000, 125, dict(bit_transition=True, sampled_ms=4, ms_per_code=4,
                                                 samples_per_code=32000.0)), (1, 1)),  # C4: 125 Hz bins
             ((8000000, 32000, 5000, 125, dict(sampled_ms=4, ms_per_code=4, samples_per_code=32000.0)), (2, 1)),
             ((25000000, 100000, 5000, 250, dict(sampled_ms=4, ms_per_code=4, samples_per_code=100000.0)), (1, 1)),
             ((4000000, 4000, 10000, 300, {}), (10, 3))]
    for (fs, N, dmax, dstep, kw), want in cases:
        acq = gsdr.Acquisition(fs, N, dmax, dstep, pfa=0.01, max_prns=1, **kw)
        assert acq.spectrum_reuse == want, (fs, N, dstep)
        acq.set_wipeoff("generic")  # a replayed protokernel is not shift-invariant: no reuse
        assert acq.spectrum_reuse == (acq.num_doppler_bins, 0)
        acq.set_wipeoff("exact")
        assert acq.spectrum_reuse == want
    # 4 Msps / 1 kHz bins, 333 Hz step: q = 1000 > D / 2 -- plain layout
    acq = gsdr.Acquisition(4000000, 4000, 5000, 333, pfa=0.01, max_prns=1)
    assert acq.spectrum_reuse == (acq.num_doppler_bins, 0)
    # a Doppler span wider than fs (step fs/2 over 5 bins: ext = 4 N/2 > N): the mirrored
    # bins would not cover the rows' windows -- plain layout
    acq = gsdr.Acquisition(2000000, 2000, 2500000, 1000000, pfa=0.01, max_prns=1)
    assert acq.num_doppler_bins == 5 and acq.spectrum_reuse == (5, 0)


@pytest.mark.parametrize("cfg_name", ["C2", "C4bt"])
def test_spectrum_reuse_is_the_plain_layout(monkeypatch, cfg_name):
    """Reused spectra vs one forward FFT per Doppler row (GSDR_ACQ_XSHIFT=0), both on
    the exact carrier: same cells, values within fp32 FFT rounding."""
    cfg = CONFIGS[cfg_name]()
    a = _acq(cfg, 0.01)
    assert a.spectrum_reuse[0] < a.num_doppler_bins
    r1 = a.run(cfg["x"])[0]
    monkeypatch.setenv("GSDR_ACQ_XSHIFT", "0")
    b = _acq(cfg, 0.01)
    assert b.spectrum_reuse == (b.num_doppler_bins, 0)
    r0 = b.run(cfg["x"])[0]
    for p in range(len(cfg["prns"])):
        assert (r1[p]["doppler_index"], r1[p]["code_phase"]) == (r0[p]["doppler_index"], r0[p]["code_phase"])
        for f in ("peak", "input_power", "test_statistic"):
            assert abs(r1[p][f] - r0[p][f]) <= 1e-5 * abs(r0[p][f]), (p, f)


@pytest.mark.parametrize("mode", ["generic", "avx2"])
@pytest.mark.parametrize("cfg_name", ["C2", "C4bt"])
def test_replayed_protokernels_match_oracle(cfg_name, mode):
    """GSDR_WIPE_GENERIC / GSDR_WIPE_AVX2: the protokernel replayed on the device, parity
    with the oracle's restatement of the same protokernel."""
    cfg = CONFIGS[cfg_name]()
    for pfa in (0.01, 0.0):
        acq = _acq(cfg, pfa, mode)
        res = acq.run(cfg["x"])[0]
        grids = _grids(cfg, acq.num_doppler_bins, mode)
        exact = sum(_check(res[p], grids[p], pfa, cfg) for p in range(len(cfg["prns"])))
        assert exact >= len(cfg["prns"]) - 1


@pytest.mark.parametrize("cfg_name", ["C2", "C3", "C4bt"])
def test_exact_carrier_vs_reference_protokernels(cfg_name):
    """The default (exact carrier, reused spectra) against the fp64 oracle at RTOL, and
    against both reference protokernels within their own distance from the exact
    carrier (+ RTOL); the spread is logged to GSDR_PARITY_LOG (tag acq_wipe)."""
    cfg = CONFIGS[cfg_name]()
    acq = _acq(cfg, 0.01)
    res = acq.run(cfg["x"])[0]
    D = acq.num_doppler_bins
    G = {m: _grids(cfg, D, m) for m in pcps.WIPE_MODES}
    worst = {"gpu_exact": 0.0, "gpu_generic": 0.0, "gpu_avx2": 0.0, "generic_exact": 0.0, "avx2_exact": 0.0,
             "generic_avx2": 0.0}
    exact_cells = 0
    for p in range(len(cfg["prns"])):
        exact_cells += _check(res[p], G["exact"][p], 0.01, cfg)
        pk = {m: float(G[m][p].max()) for m in pcps.WIPE_MODES}
        g = float(res[p]["peak"])
        e = pk["exact"]
        for m in ("generic", "avx2"):
            assert abs(g - pk[m]) <= abs(pk[m] - e) + RTOL * e, (p, m, g, pk)
            worst["gpu_" + m] = max(worst["gpu_" + m], abs(g - pk[m]) / e)
            worst[m + "_exact"] = max(worst[m + "_exact"], abs(pk[m] - e) / e)
        worst["gpu_exact"] = max(worst["gpu_exact"], abs(g - e) / e)
        worst["generic_avx2"] = max(worst["generic_avx2"], abs(pk["generic"] - pk["avx2"]) / e)
    _log({"tag": "acq_wipe", "config": cfg_name, "N": cfg["N"], "prns": len(cfg["prns"]),
          "reuse": list(acq.spectrum_reuse), "exact_cells": int(exact_cells),
          "peak_rel_max": {k: float("%.3g" % v) for k, v in worst.items()}})
    assert exact_cells >= len(cfg["prns"]) - 1


def test_grid_dump_with_reuse_at_split_size():
    """gsdr_acq_dump_grid (the reference's dump grid, pcps_acquisition.cc:408-508) at a
    split size with reused spectra (C5 GPS: N = 25000, 4 spectra per block) against the
    oracle's exact-carrier grid."""
    fs, N, dmax, dstep = 25000000, 25000, 10000, 250
    sats = synth.random_constellation(4, seed_offset=41)
    x = synth.gps_l1_iq(fs, N, sats, seed_offset=41)
    prns = np.array([sats[0].prn, 32])
    codes = np.stack([synth.gps_ca_sampled(int(p), fs, N) for p in prns])
    acq = gsdr.Acquisition(fs, N, dmax, dstep, pfa=0.01, max_prns=2)
    acq.set_local_codes(codes, prns)
    assert acq.spectrum_reuse == (4, 1)
    g = acq.dump_grid(x, 0)
    wipe = pcps.doppler_wipeoffs(fs, N, dmax, dstep, acq.num_doppler_bins)
    M = pcps.magnitude_grid(x, wipe, pcps.fft_code(codes[0], N, N))
    assert np.max(np.abs(g - M)) <= 1e-5 * M.max()
