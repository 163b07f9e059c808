"""GPU parity of make_two_steps (pcps_acquisition.cc:298-314 narrow grid, :717-773
second step, :781-800 decision, :894-909 threshold) against the oracle restatement.

The first step runs the full grid on block 0; every PRN it declares positive is
refined on block 1 on num_doppler_bins_step2 bins spaced doppler_step2 around its
coarse Acq_doppler_hz, the CFAR statistic dividing by the first step's input power.
Tolerances as tests/test_gpu_acq.py: cells equal (or a 1e-4 near tie), peak and
statistic within 1e-4 relative, Doppler and thresholds exact.
"""
import numpy as np
import pytest

import gsdr
from gsdr import synth
from oracle import pcps

pytestmark = pytest.mark.gpu

RTOL = 1e-4


def _run_two_steps(fs, N, pfa, nbins2, step2, pfa2=0.0, prns=None, seed=11):
    sats = synth.random_constellation(6, seed_offset=seed, cn0_dbhz=48.0)
    x = synth.gps_l1_iq(fs, 2 * N, sats, seed_offset=seed)
    x0, x1 = x[:N], x[N:]
    prns = np.array([s.prn for s in sats] + [p for p in (31, 32) if p not in [s.prn for s in sats]][:2])
    codes = np.stack([synth.gps_ca_sampled(int(p), fs, N) for p in prns])
    dmax, dstep = 10000, 500
    acq = gsdr.Acquisition(fs, N, dmax, dstep, pfa=pfa, max_prns=len(prns))
    acq.set_local_codes(codes, prns)
    acq.set_step_two(nbins2, step2, pfa2)
    coarse = acq.run(x0)[0]
    sel = np.nonzero(coarse["positive"])[0] if pfa > 0 else np.argsort(-coarse["test_statistic"])[:4]
    assert len(sel) >= 2, coarse
    fine = acq.run_step_two(x1, sel, coarse["doppler_hz"][sel].astype(np.float32),
                            coarse["input_power"][sel], stamp=N)
    return acq, sats, prns, codes, x1, coarse, sel, fine


def _check(acq, sats, prns, codes, x1, coarse, sel, fine, fs, N, pfa, nbins2, step2, pfa2):
    spc = int(np.ceil(fs / 1023000.0))
    thr1 = pcps.threshold(pfa, N, acq.num_doppler_bins) if pfa > 0 else acq.threshold
    thr2 = pcps.threshold_step_two(pfa, pfa2, N, nbins2, first_threshold=thr1)
    assert acq.step_two_threshold == pytest.approx(thr2, rel=1e-6)
    true_dop = {s.prn: s.doppler_hz for s in sats}
    improved = 0
    for i, slot in enumerate(sel):
        r = fine[i]
        center = np.float32(coarse["doppler_hz"][slot])
        wipe = pcps.doppler_wipeoffs_step2(fs, N, center, step2, nbins2)
        M = pcps.magnitude_grid(x1, wipe, pcps.fft_code(codes[slot], N, N))
        ti, di, gmax, second, stat, dop = pcps.step_two_statistic(
            M, coarse["input_power"][slot], center, step2, spc, N, cfar=pfa > 0)
        assert int(r["prn"]) == int(prns[slot])
        assert int(r["samplestamp"]) == N
        if (int(r["doppler_index"]), int(r["code_phase"])) != (di, ti):
            assert abs(M[r["doppler_index"], r["code_phase"]] - gmax) <= RTOL * gmax, (r, di, ti)
            continue
        assert abs(float(r["peak"]) - float(gmax)) <= RTOL * float(gmax)
        assert int(r["doppler_hz"]) == dop
        assert abs(float(r["test_statistic"]) - float(stat)) <= RTOL * float(stat)
        if pfa > 0:
            assert float(r["input_power"]) == float(coarse["input_power"][slot])
        else:
            assert abs(float(r["second_peak"]) - float(second)) <= RTOL * float(second)
        assert int(r["positive"]) == int(float(r["test_statistic"]) > thr2)
        p = int(prns[slot])
        if p in true_dop and abs(dop - true_dop[p]) < abs(int(coarse["doppler_hz"][slot]) - true_dop[p]):
            improved += 1
    return improved


@pytest.mark.parametrize("fs,pfa,pfa2", [(4000000, 0.01, 0.0), (4000000, 0.01, 0.001), (3000000, 0.01, 0.0),
                                         (4000000, 0.0, 0.0), (25000000, 0.01, 0.0), (25000000, 0.0, 0.0)])
def test_two_steps_parity(fs, pfa, pfa2):
    """25 Msps: N = 25000 on the split register four-step (coarse grid with two reused
    forward spectra, the narrow grid's selected rows on the split plan)."""
    N = fs // 1000
    nbins2, step2 = 5, 100.0
    out = _run_two_steps(fs, N, pfa, nbins2, step2, pfa2)
    improved = _check(*out, fs, N, pfa, nbins2, step2, pfa2)
    if pfa > 0:
        assert improved >= 1  # the refinement moves some estimate towards the truth


def test_two_steps_even_bins_and_fractional_step():
    fs, N = 4000000, 4000
    out = _run_two_steps(fs, N, 0.01, 4, 62.5, 0.0, seed=5)
    _check(*out, fs, N, 0.01, 4, 62.5, 0.0)


def test_two_steps_argument_errors():
    fs, N = 4000000, 4000
    acq = gsdr.Acquisition(fs, N, 5000, 500, pfa=0.01, max_prns=2)
    acq.set_local_codes(np.stack([synth.gps_ca_sampled(p, fs, N) for p in (1, 2)]), np.array([1, 2]))
    x = np.zeros(N, np.complex64)
    with pytest.raises(gsdr.GsdrError):
        acq.run_step_two(x, [0], [0.0], [1.0])  # set_step_two first
    acq.set_step_two(4, 125.0)
    with pytest.raises(gsdr.GsdrError):
        acq.run_step_two(x, [2], [0.0], [1.0])  # slot outside the batch
