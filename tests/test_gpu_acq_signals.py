"""GPU acquisition parity for Galileo E1 and BeiDou B1I (SURVEY §8 a3, configs C4/C5
replicas) against the oracle, through the C ABI.  Same tolerances as
test_gpu_acq.py (1e-4 relative, equal cells or H3 near ties)."""
import os

import numpy as np
import pytest

import gsdr
from conftest import GOLDEN
from gsdr import synth
from oracle import pcps, replica
from test_gpu_acq import _check_result, _oracle_grids

pytestmark = pytest.mark.gpu


def test_galileo_reference_capture():
    """galileo_e1_pcps_ambiguous_acquisition_test.cc:295-370 on the GPU: PRN 1 E1B,
    4 Msps, N = 16000 (4 ms), +-10 kHz / 250 Hz, pfa 0.001."""
    x = np.fromfile(os.path.join(GOLDEN, "Galileo_E1_ID_1_Fs_4Msps_8ms.dat"), np.complex64)
    fs, dmax, dstep = 4000000, 10000, 250
    code = replica.galileo_e1_code_complex_sampled("1B", False, 1, fs)
    acq = gsdr.Acquisition(fs, 16000, dmax, dstep, pfa=0.001, max_prns=1, max_blocks=2, sampled_ms=4, ms_per_code=4)
    assert acq.fft_size == 16000 and acq.num_doppler_bins == 80
    acq.set_local_codes(code[None, :], [1])
    res = acq.run(x, nblocks=2)
    r = res[0, 0]
    assert r["positive"] == 1
    assert abs(2920 - r["acq_delay_samples"]) * 1023 / fs < 0.175
    assert abs(-632 - r["doppler_hz"]) <= 166
    for b in range(2):
        M = _oracle_grids(x[b * 16000:(b + 1) * 16000], [code], fs, dmax, dstep, 80)[0]
        _check_result(res[b, 0], M, 0.001, 4, fs, dmax, dstep, 16000.0)


@pytest.mark.parametrize("cboc", [False, True])
def test_galileo_e1_synthetic_batch(cboc):
    """E1 at 4 Msps, one 4 ms code period per block (N = 16000), 10 PRNs, 4 visible."""
    fs, N, dmax, dstep = 4000000, 16000, 5000, 250
    rng = np.random.default_rng(4)
    vis = [2, 9, 21, 30]
    sats = [synth.GalileoSatellite(p, float(rng.uniform(-4000, 4000)), float(rng.uniform(0, 4092)), 50.0,
                                   float(rng.uniform(0, 6.28))) for p in vis]
    x = synth.gal_e1_iq(fs, N, sats, seed_offset=4)
    prns = np.array([2, 3, 9, 11, 17, 21, 25, 30, 33, 36])
    codes = np.stack([synth.gal_e1_sampled(int(p), fs, cboc=cboc) for p in prns])
    acq = gsdr.Acquisition(fs, N, dmax, dstep, pfa=0.01, max_prns=len(prns), sampled_ms=4, ms_per_code=4)
    assert acq.fft_size == N
    acq.set_local_codes(codes, prns)
    res = acq.run(x)[0]
    D = acq.num_doppler_bins
    grids = _oracle_grids(x, codes, fs, dmax, dstep, D)
    spc = int(np.ceil(fs / 1023000.0))
    exact = sum(_check_result(res[i], grids[i], 0.01, spc, fs, dmax, dstep, 16000.0) for i in range(len(prns)))
    assert exact >= len(prns) - 1
    # detection (not parity): 4 ms coherent with up to 125 Hz grid mismatch loses up to 3.9 dB
    det = {int(r["prn"]) for r in res if r["positive"]}
    assert len(set(vis) & det) >= 3


@pytest.mark.parametrize("fs", [6000000, 10000000])
def test_beidou_b1i_synthetic_batch(fs):
    """B1I (2.046 Mcps, 1 ms code): 12 PRNs, 5 visible, +-5 kHz / 250 Hz."""
    N = fs // 1000
    dmax, dstep = 5000, 250
    rng = np.random.default_rng(fs // 1000000)
    vis = [1, 6, 14, 33, 59]
    sats = [synth.Satellite(p, float(rng.uniform(-4000, 4000)), float(rng.uniform(0, 2046)), 50.0,
                            float(rng.uniform(0, 6.28))) for p in vis]
    x = synth.bds_b1i_iq(fs, N, sats, seed_offset=1)
    prns = np.array([1, 2, 6, 8, 14, 20, 27, 33, 40, 50, 59, 63])
    codes = np.stack([synth.bds_b1i_sampled(int(p), fs) for p in prns])
    acq = gsdr.Acquisition(fs, N, dmax, dstep, pfa=0.01, max_prns=len(prns), chip_rate=2046000.0)
    acq.set_local_codes(codes, prns)
    res = acq.run(x)[0]
    grids = _oracle_grids(x, codes, fs, dmax, dstep, acq.num_doppler_bins)
    spc = int(np.ceil(fs / 2046000.0))
    exact = sum(_check_result(res[i], grids[i], 0.01, spc, fs, dmax, dstep, float(N)) for i in range(len(prns)))
    assert exact >= len(prns) - 1
    det = {int(r["prn"]) for r in res if r["positive"]}
    assert set(vis) <= det


LARGE_CONFIGS = [(8000000, 32000, 0.01), (25000000, 25000, 0.0), (8000000, 64000, 0.01), (25000000, 100000, 0.01),
                 (25000000, 25000, 0.01), (25000000, 100000, 0.0)]


def _split_cases():
    """Every configuration on both correlate paths."""
    return [(fs, n, pfa, split) for fs, n, pfa in LARGE_CONFIGS for split in ("1", "0")]


@pytest.mark.parametrize("fs,N,pfa,split", _split_cases())
def test_large_fft_four_step(monkeypatch, fs, N, pfa, split):
    """N beyond one workgroup's LDS: Galileo E1 at 8 Msps (4 ms: 32000; 8 ms:
    64000), BeiDou B1I at 25 Msps (1 ms: 25000), Galileo at 25 Msps (100000) --
    configs C4/C5 -- on both correlate paths: GSDR_ACQ_SPLIT=1 (default: the split
    register four-step for 25000 / 32000 / 64000 / 100000 = 4 x 25000) and 0 (the
    packed four-step everywhere).  Parity with the oracle grid statistics."""
    monkeypatch.setenv("GSDR_ACQ_SPLIT", split)
    dmax, dstep = 2000, 500
    rng = np.random.default_rng(N)
    if N == 25000:
        sats = [synth.Satellite(p, float(rng.uniform(-1500, 1500)), float(rng.uniform(0, 2046)), 50.0, 0.3)
                for p in (3, 11)]
        x = synth.bds_b1i_iq(fs, N, sats, seed_offset=2)
        prns = np.array([3, 5, 11])
        codes = np.stack([synth.bds_b1i_sampled(int(p), fs) for p in prns])
        chip, spcode, ms = 2046000.0, float(N), 1
    else:
        sats = [synth.GalileoSatellite(p, float(rng.uniform(-1500, 1500)), float(rng.uniform(0, 4092)), 50.0, 0.3)
                for p in (4, 19)]
        x = synth.gal_e1_iq(fs, N, sats, seed_offset=2)
        prns = np.array([4, 7, 19])
        one = [synth.gal_e1_sampled(int(p), fs) for p in prns]
        codes = np.stack([np.resize(c, N) for c in one])
        chip, spcode, ms = 1023000.0, float(len(one[0])), N * 1000 // fs
    acq = gsdr.Acquisition(fs, N, dmax, dstep, pfa=pfa, max_prns=len(prns), chip_rate=chip, sampled_ms=ms,
                           ms_per_code=ms, samples_per_code=spcode)
    assert acq.fft_size == N
    acq.set_local_codes(codes, prns)
    res = acq.run(x)[0]
    grids = _oracle_grids(x, codes, fs, dmax, dstep, acq.num_doppler_bins)
    spc = int(np.ceil(fs / chip))
    for i in range(len(prns)):
        _check_result(res[i], grids[i], pfa, spc, fs, dmax, dstep, spcode)
    # the forward spectra themselves (first Doppler row)
    X = acq.dump_spectra(x)
    ref = np.fft.fft(x.astype(np.complex128) * pcps.doppler_wipeoffs(fs, N, dmax, dstep, acq.num_doppler_bins)[0])
    assert np.linalg.norm(X[0] - ref) / np.linalg.norm(ref) < 2e-6
