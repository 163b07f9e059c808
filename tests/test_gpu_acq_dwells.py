"""GPU parity of acquisition_core's non-coherent dwells (max_dwells > 1) and
bit-transition mode (pcps_acquisition.cc:615-882) against the
oracle, through the C ABI.  Per attempt and PRN the reported result is the first
dwell whose statistic crosses the threshold, else the last (:781-869)."""
import numpy as np
import pytest

import gsdr
from gsdr import synth
from oracle import pcps

pytestmark = pytest.mark.gpu

RTOL = 1e-4
FS, C = 4000000, 4000


def _oracle_attempt(chunks, codes, pfa, D, dmax, dstep, bit_transition, spc, threshold, fs=FS):
    """Per PRN: (dwell index, ti, di, peak, input_power/second, stat) of the decision."""
    N = len(chunks[0])
    wipe = pcps.doppler_wipeoffs(fs, N, dmax, dstep, D)
    out = []
    for code in codes:
        cf = pcps.fft_code(code, N, N, bit_transition=bit_transition)
        acc = None
        for k, x in enumerate(chunks):
            M = pcps.magnitude_grid(x, wipe, cf, bit_transition=bit_transition)
            acc = M if acc is None else (acc + M).astype(np.float32)
            if pfa > 0:
                ti, di, peak, ip, stat = pcps.max_to_input_power_statistic(acc, k + 1)
                aux = ip
            else:
                full = np.zeros((D, N), np.float32)
                full[:, :acc.shape[1]] = acc
                ti, di, peak, aux, stat = pcps.first_vs_second_peak_statistic(full, spc, N)
            if stat > threshold or k + 1 == len(chunks):
                out.append((k, ti, di, peak, aux, stat, acc))
                break
    return out


def _check(r, o, pfa):
    k, ti, di, peak, aux, stat, acc = o
    assert r["num_dwells"] == k + 1
    if (r["doppler_index"], r["code_phase"]) != (di, ti):  # near tie
        assert abs(acc[r["doppler_index"], r["code_phase"]] - peak) <= RTOL * peak
        return
    assert abs(r["peak"] - peak) <= RTOL * peak
    assert abs(r["test_statistic"] - stat) <= RTOL * stat
    if pfa > 0:
        assert abs(r["input_power"] - aux) <= RTOL * aux
    else:
        assert abs(r["second_peak"] - aux) <= RTOL * aux


@pytest.mark.parametrize("pfa", [0.01, 0.0])
def test_noncoherent_dwells(pfa):
    K, nat, dmax, dstep = 3, 2, 5000, 500
    sats = synth.random_constellation(6, seed_offset=11, cn0_dbhz=44.0, max_doppler=4500.0)
    x = synth.gps_l1_iq(FS, nat * K * C, sats, seed_offset=11)
    prns = np.array([s.prn for s in sats] + [31, 32])
    codes = np.stack([synth.gps_ca_sampled(int(p), FS) for p in prns])
    acq = gsdr.Acquisition(FS, C, dmax, dstep, pfa=pfa, max_prns=len(prns), max_blocks=nat, max_dwells=K)
    acq.set_local_codes(codes, prns)
    thr = pcps.threshold(pfa, C, acq.num_doppler_bins, K) if pfa > 0 else 2.5
    if pfa > 0:
        assert abs(acq.threshold - thr) <= 1e-6 * thr
    else:
        acq.set_threshold(thr)
    res = acq.run(x, nblocks=nat, stamp0=100)
    used = set()
    for a in range(nat):
        chunks = [x[(a * K + k) * C:(a * K + k + 1) * C] for k in range(K)]
        orc = _oracle_attempt(chunks, codes, pfa, acq.num_doppler_bins, dmax, dstep, False, 4, thr)
        for i in range(len(prns)):
            r = res[a, i]
            _check(r, orc[i], pfa)
            assert r["samplestamp"] == 100 + (a * K + orc[i][0]) * C
            assert r["positive"] == int(orc[i][5] > thr)
            used.add(int(r["num_dwells"]))
    assert len(used) >= 2  # some decisions before the last dwell, some at it


@pytest.mark.parametrize("pfa", [0.01, 0.0])
def test_bit_transition(pfa):
    """bit_transition_flag: consumed = 2 x 1 ms, FFT 8000 with the code in the
    second half, outputs [4000, 8000), threshold on 4000 x D cells, one dwell."""
    dmax, dstep = 5000, 250
    sats = synth.random_constellation(5, seed_offset=12, cn0_dbhz=45.0, max_doppler=4500.0)
    nb = 2
    x = synth.gps_l1_iq(FS, nb * 2 * C, sats, seed_offset=12)
    prns = np.array([s.prn for s in sats] + [30])
    codes = np.stack([np.resize(synth.gps_ca_sampled(int(p), FS), 2 * C) for p in prns])
    acq = gsdr.Acquisition(FS, 2 * C, dmax, dstep, pfa=pfa, max_prns=len(prns), max_blocks=nb, bit_transition=True,
                           max_dwells=4)
    assert acq.fft_size == 2 * C
    acq.set_local_codes(codes, prns)
    D = acq.num_doppler_bins
    thr = pcps.threshold(pfa, 2 * C, D, 4, bit_transition=True) if pfa > 0 else 2.0
    if pfa > 0:
        assert abs(acq.threshold - thr) <= 1e-6 * thr
    else:
        acq.set_threshold(thr)
    res = acq.run(x, nblocks=nb)
    for b in range(nb):
        chunk = x[b * 2 * C:(b + 1) * 2 * C]
        orc = _oracle_attempt([chunk], codes, pfa, D, dmax, dstep, True, 4, thr)
        for i in range(len(prns)):
            _check(res[b, i], orc[i], pfa)
            assert res[b, i]["samplestamp"] == b * 2 * C


@pytest.mark.parametrize("split", ["1", "0"])
@pytest.mark.parametrize("pfa", [0.01, 0.0])
def test_bit_transition_c4_four_step(monkeypatch, pfa, split):
    """Config C4's acquisition as the bench times it (pcps_acquisition.cc:85-92,
    :188-193, :671): Galileo E1 at 8 Msps, 4 ms code, bit_transition_flag -> FFT
    64000 with the code in the second half and outputs [32000, 64000), +-10 kHz /
    250 Hz (80 bins): the split register four-step (default: ROUT = 2 over a
    32000-point wave-local-row register transform, row maxima of outputs k >= N/2,
    acq_split.hip id 13) and the general (dwell) path over the packed four-step
    (GSDR_ACQ_SPLIT=0)."""
    monkeypatch.setenv("GSDR_ACQ_SPLIT", split)
    fs, C, dmax, dstep = 8000000, 32000, 10000, 250
    rng = np.random.default_rng(64)
    vis = [4, 19]
    sats = [synth.GalileoSatellite(p, float(rng.uniform(-8000, 8000)), float(rng.uniform(0, 4092)), 47.0,
                                   float(rng.uniform(0, 6.28))) for p in vis]
    x = synth.gal_e1_iq(fs, 2 * C, sats, seed_offset=64)
    prns = np.array([4, 7, 19, 30])
    codes = np.stack([np.resize(synth.gal_e1_sampled(int(p), fs), 2 * C) for p in prns])
    acq = gsdr.Acquisition(fs, 2 * C, dmax, dstep, pfa=pfa, max_prns=len(prns), bit_transition=True, sampled_ms=4,
                           ms_per_code=4, samples_per_code=float(C))
    assert acq.fft_size == 2 * C and acq.num_doppler_bins == 80
    acq.set_local_codes(codes, prns)
    D = acq.num_doppler_bins
    spc = int(np.ceil(fs / 1023000.0))
    thr = pcps.threshold(pfa, 2 * C, D, 1, bit_transition=True) if pfa > 0 else 2.0
    if pfa > 0:
        assert abs(acq.threshold - thr) <= 1e-6 * thr
    else:
        acq.set_threshold(thr)
    res = acq.run(x)
    orc = _oracle_attempt([x], codes, pfa, D, dmax, dstep, True, spc, thr, fs=fs)
    for i in range(len(prns)):
        _check(res[0, i], orc[i], pfa)
        assert res[0, i]["positive"] == int(orc[i][5] > thr)
    if pfa > 0:  # detection (not parity)
        assert {int(r["prn"]) for r in res[0] if r["positive"]} >= set(vis)


@pytest.mark.parametrize("pfa", [0.01, 0.0])
def test_noncoherent_dwells_four_step(pfa):
    """max_dwells > 1 at a four-step size (Galileo E1, 8 Msps, 4 ms: N = 32000):
    the dwell accumulator rows of the general path on the packed four-step."""
    fs, C, K, dmax, dstep = 8000000, 32000, 2, 3000, 500
    rng = np.random.default_rng(32)
    sats = [synth.GalileoSatellite(p, float(rng.uniform(-2500, 2500)), float(rng.uniform(0, 4092)), 43.0,
                                   float(rng.uniform(0, 6.28))) for p in (4, 19)]
    x = synth.gal_e1_iq(fs, K * C, sats, seed_offset=32)
    prns = np.array([4, 7, 19])
    codes = np.stack([synth.gal_e1_sampled(int(p), fs) for p in prns])
    acq = gsdr.Acquisition(fs, C, dmax, dstep, pfa=pfa, max_prns=len(prns), max_dwells=K, sampled_ms=4,
                           ms_per_code=4, samples_per_code=float(C))
    assert acq.fft_size == C
    acq.set_local_codes(codes, prns)
    D = acq.num_doppler_bins
    spc = int(np.ceil(fs / 1023000.0))
    thr = pcps.threshold(pfa, C, D, K) if pfa > 0 else 3.0
    if pfa > 0:
        assert abs(acq.threshold - thr) <= 1e-6 * thr
    else:
        acq.set_threshold(thr)
    res = acq.run(x, stamp0=7)
    chunks = [x[k * C:(k + 1) * C] for k in range(K)]
    orc = _oracle_attempt(chunks, codes, pfa, D, dmax, dstep, False, spc, thr, fs=fs)
    for i in range(len(prns)):
        _check(res[0, i], orc[i], pfa)
        assert res[0, i]["samplestamp"] == 7 + orc[i][0] * C
        assert res[0, i]["positive"] == int(orc[i][5] > thr)
