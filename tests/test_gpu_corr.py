"""GPU parity of the fused tracking multicorrelator against the oracle
(VOLK-GNSSSDR generic resampler + rotator dot product), through the C ABI.

- Code-phase indices: bit-exact, for both float associations (generic / a_avx).
- Taps vs the reference generic kernel: ccompare <= 1e-4 per tap (north_star fp32 tolerance).
- Taps vs the fp64 evaluation of the same phasor model: vector-norm relative <= 1e-5
  (the GPU is closer to exact than the generic kernel).
"""
import numpy as np
import pytest
import torch

import gsdr
from gsdr import synth
from oracle import volk

from conftest import ccompare, vnorm_rel

pytestmark = pytest.mark.gpu


def _signal(fs, N, prn, doppler, delay_chips, cn0=55.0, seed=0, code=None):
    sats = [synth.Satellite(prn, doppler, delay_chips, cn0)]
    return synth.gps_l1_iq(fs, N, sats, seed_offset=seed)


def _galileo_code(prn=11):
    """Galileo E1-B tracking replica: the ICD memory code as sinBOC(1,1) at 2 samples
    per chip (galileo_e1_code_gen_sinboc11_float, galileo_e1_signal_replica.cc:100-111)."""
    return synth.gal_e1_sinboc11(prn).astype(np.float32)


@pytest.mark.parametrize("assoc", [gsdr.ASSOC_GENERIC, gsdr.ASSOC_AVX])
@pytest.mark.parametrize("L", [1023, 8184])
def test_indices_bit_exact(assoc, L):
    corr = gsdr.Correlator(1, 40000, max_taps=5)
    corr.set_resampler_assoc(assoc)
    shifts = np.array([-0.6, -0.15, 0.0, 0.15, 0.6], np.float32) * (2 if L == 8184 else 1)
    corr.set_local_code_and_taps(0, np.ones(L, np.float32), shifts)
    rng = np.random.default_rng(L + assoc)
    for trial in range(8):
        N = 32000 if L == 8184 else 16000
        rem = float(rng.uniform(-0.5, 0.5))
        step = float(np.float32(L / N * (1 + rng.uniform(-3e-6, 3e-6))))
        got = corr.dump_indices(0, rem, step, N)
        ref = volk.resampler_index(rem, step, shifts, L, N, assoc=assoc)
        np.testing.assert_array_equal(got, ref)


CASES = [
    # name, fs, N, L, spc, shifts (chips)
    ("gps_c1_k3", 4e6, 4000, 1023, 1, [-0.5, 0.0, 0.5]),
    ("gps_c3_k5", 16e6, 16000, 1023, 1, [-0.5, -0.25, 0.0, 0.25, 0.5]),
    ("gal_c4_k5", 8e6, 32000, 8184, 2, [-0.6, -0.15, 0.0, 0.15, 0.6]),
]


@pytest.mark.parametrize("name,fs,N,L,spc,shifts_chips", CASES)
def test_taps_vs_generic_and_exact(name, fs, N, L, spc, shifts_chips):
    code = synth.gps_ca_chips(5) if L == 1023 else _galileo_code()
    shifts = np.array(shifts_chips, np.float32) * spc
    corr = gsdr.Correlator(2, N, max_taps=8)
    corr.set_local_code_and_taps(0, code, shifts)
    corr.set_local_code_and_taps(1, code, shifts[len(shifts) // 2:len(shifts) // 2 + 1])  # data-prompt tap
    rng = np.random.default_rng(N)
    doppler = 1523.25
    for trial in range(3):
        if L == 1023:
            x = _signal(fs, N, 5, doppler, 0.0, seed=trial)
        else:
            x = (rng.standard_normal(N) + 1j * rng.standard_normal(N)).astype(np.complex64)
            t = np.arange(N) / fs
            x += (3.0 * code[(np.floor(t * 2.046e6)).astype(np.int64) % L] *
                  np.exp(2j * np.pi * doppler * t)).astype(np.complex64)
        rem_carr = float(np.float32(rng.uniform(-np.pi, np.pi)))
        carr_step = float(np.float32(2 * np.pi * doppler / fs))
        rem_code = float(np.float32(rng.uniform(-0.1, 0.1) * spc))
        code_step = float(np.float32(1.023e6 * spc / fs * (1 + 1e-7)))
        got = corr.run(0, x, rem_carr, carr_step, rem_code, code_step, N)
        gen = volk.multicorrelator_real_codes(x, code, shifts, rem_carr, carr_step, rem_code, code_step, N)
        exact = volk.multicorrelator_real_codes_exact(x, code, shifts, rem_carr, carr_step, rem_code, code_step, N)
        assert ccompare(got, gen) <= 1e-4, (name, got, gen)
        assert vnorm_rel(got, exact) <= 1e-5, (name, got, exact)
        d = corr.run(1, x, rem_carr, carr_step, rem_code, code_step, N)
        assert ccompare(d, got[len(shifts) // 2:len(shifts) // 2 + 1]) <= 1e-6


def test_uniform_noise_input_like_reference_timing_test():
    """cpu_multicorrelator_real_codes_test.cc inputs: uniform(0,1) IQ, phase step 0.1 rad."""
    rng = np.random.default_rng(7)
    N = 8192
    x = (rng.uniform(0, 1, N) + 1j * rng.uniform(0, 1, N)).astype(np.complex64)
    code = synth.gps_ca_chips(1)
    shifts = np.array([-0.5, 0.0, 0.5], np.float32)
    corr = gsdr.Correlator(1, N, max_taps=3)
    corr.set_local_code_and_taps(0, code, shifts)
    got = corr.run(0, x, 0.0, 0.1, 0.4, 0.3, N)
    exact = volk.multicorrelator_real_codes_exact(x, code, shifts, 0.0, 0.1, 0.4, 0.3, N)
    gen = volk.multicorrelator_real_codes(x, code, shifts, 0.0, 0.1, 0.4, 0.3, N)
    assert vnorm_rel(got, exact) <= 1e-5
    assert vnorm_rel(got, gen) <= 1e-3  # noise-only taps: the generic kernel's own fp32 error dominates


def test_complex_codes():
    """Cpu_Multicorrelator (complex replicas, cpu_multicorrelator.cc:73-100)."""
    fs, N = 4e6, 4000
    code = synth.gps_ca_sampled(9, 1023000).astype(np.complex64)  # (0, +-1), one sample per chip
    code = (code + 0.5 * np.roll(code, 3).imag).astype(np.complex64)
    shifts = np.array([-0.5, 0.0, 0.5], np.float32)
    x = _signal(fs, N, 9, -800.0, 12.0, seed=3)
    corr = gsdr.Correlator(1, N, max_taps=3)
    corr.set_local_code_and_taps(0, code, shifts)
    args = (0.7, float(np.float32(2 * np.pi * -800.0 / fs)), 0.2, float(np.float32(1.023e6 / fs)))
    got = corr.run(0, x, *args, N)
    ref = volk.multicorrelator_complex_codes(x, code, shifts, *args, N)
    assert ccompare(got, ref) <= 1e-4


def test_high_dynamics_resampler_and_rotator():
    fs, N = 4e6, 4000
    code = synth.gps_ca_chips(11)
    shifts = np.array([-0.5, 0.0, 0.5], np.float32)
    x = _signal(fs, N, 11, 2100.0, 40.0, seed=4)
    corr = gsdr.Correlator(1, N, max_taps=3)
    corr.set_local_code_and_taps(0, code, shifts)
    corr.set_high_dynamics_resampler(0, True)
    rem_carr, carr_step, carr_rate = 0.1, float(np.float32(2 * np.pi * 2100.0 / fs)), 2e-9
    rem_code, code_step, code_rate = 0.3, float(np.float32(1.023e6 / fs)), 1e-10
    got = corr.run(0, x, rem_carr, carr_step, rem_code, code_step, N, carr_rate=carr_rate, code_rate=code_rate)
    ref = volk.multicorrelator_real_codes(x, code, shifts, rem_carr, carr_step, rem_code, code_step, N,
                                          carr_rate=carr_rate, code_rate=code_rate, high_dyn=True)
    assert ccompare(got, ref) <= 1e-4


@pytest.mark.parametrize("item_type", [gsdr.ITEM_GR_COMPLEX, gsdr.ITEM_CSHORT, gsdr.ITEM_IBYTE])
def test_batched_channels_from_device_buffer(item_type):
    """Config C3 shape: 12 channels x N=16000 x K=5 in one launch over a device IQ buffer."""
    fs, N, K = 16e6, 16000, 5
    sats = synth.random_constellation(12, seed_offset=21, prns=list(range(1, 13)))
    total = N * 3
    x = synth.gps_l1_iq(fs, total, sats, seed_offset=21)
    shifts = np.array([-0.5, -0.25, 0.0, 0.25, 0.5], np.float32)
    corr = gsdr.Correlator(12, N, max_taps=K)
    for ch, s in enumerate(sats):
        corr.set_local_code_and_taps(ch, synth.gps_ca_chips(s.prn), shifts)
    rng = np.random.default_rng(5)
    jobs = np.zeros(12, gsdr.CORR_JOB_DTYPE)
    for ch, s in enumerate(sats):
        jobs[ch] = (ch, N - int(rng.integers(0, 3)), int(rng.integers(0, N)),
                    np.float32(rng.uniform(-3, 3)), np.float32(2 * np.pi * s.doppler_hz / fs), 0.0,
                    np.float32(rng.uniform(-0.5, 0.5)), np.float32(1.023e6 / fs), 0.0)
    if item_type == gsdr.ITEM_CSHORT:
        host = synth.to_cshort(x, 1000.0)
        xf = (host[0::2].astype(np.float32) + 1j * host[1::2].astype(np.float32)).astype(np.complex64)
    elif item_type == gsdr.ITEM_IBYTE:
        host = synth.to_ibyte(x, 20.0)
        xf = synth.ibyte_to_complex(host)
    else:
        host = x
        xf = x
    dev = torch.from_numpy(host if item_type != gsdr.ITEM_GR_COMPLEX else host.view(np.float32)).cuda()
    out = torch.zeros(12 * K * 2, dtype=torch.float32, device="cuda")
    corr.run_batch(jobs, dev.data_ptr(), total, out.data_ptr(), item_type=item_type)
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.complex64).reshape(12, K)
    for ch, s in enumerate(sats):
        j = jobs[ch]
        seg = xf[j["sample_offset"]:j["sample_offset"] + j["n_samples"]]
        ref = volk.multicorrelator_real_codes(seg, synth.gps_ca_chips(s.prn), shifts, float(j["rem_carr_phase_rad"]),
                                              float(j["carr_phase_step_rad"]), float(j["rem_code_phase_chips"]),
                                              float(j["code_phase_step_chips"]), int(j["n_samples"]))
        exact = volk.multicorrelator_real_codes_exact(seg, synth.gps_ca_chips(s.prn), shifts,
                                                      float(j["rem_carr_phase_rad"]), float(j["carr_phase_step_rad"]),
                                                      float(j["rem_code_phase_chips"]),
                                                      float(j["code_phase_step_chips"]), int(j["n_samples"]))
        assert vnorm_rel(o[ch], exact) <= 1e-5
        assert vnorm_rel(o[ch], ref) <= 1e-3  # mostly noise taps here: bounded by the generic kernel's fp32 error


@pytest.mark.parametrize("N", [1, 100, 1023, 1024, 1025, 5000, 20000])
def test_chunk_boundaries(N):
    """Jobs shorter than, equal to and straddling the per-workgroup chunk."""
    fs = 4e6
    code = synth.gps_ca_chips(2)
    shifts = np.array([-0.5, 0.0, 0.5], np.float32)
    x = _signal(fs, max(N, 1), 2, 900.0, 0.0, seed=N)
    corr = gsdr.Correlator(1, 20000, max_taps=3)
    corr.set_local_code_and_taps(0, code, shifts)
    args = (0.2, float(np.float32(2 * np.pi * 900.0 / fs)), 0.05, float(np.float32(1.023e6 / fs)))
    got = corr.run(0, x, *args, N)
    exact = volk.multicorrelator_real_codes_exact(x, code, shifts, *args, N)
    assert vnorm_rel(got, exact) <= 1e-5


def test_run_epochs_matches_per_epoch_batches():
    """gsdr_corr_run_epochs: n_epochs launches in order over one job table."""
    fs, N, C, E = 4e6, 4000, 4, 6
    sats = synth.random_constellation(C, seed_offset=31)
    x = synth.gps_l1_iq(fs, N * (E + 1), sats, seed_offset=31)
    shifts = np.array([-0.5, 0.0, 0.5], np.float32)
    corr = gsdr.Correlator(C, N, max_taps=3)
    for c, s in enumerate(sats):
        corr.set_local_code_and_taps(c, synth.gps_ca_chips(s.prn), shifts)
    jobs = np.zeros(C * E, gsdr.CORR_JOB_DTYPE)
    for e in range(E):
        for c, s in enumerate(sats):
            jobs[e * C + c] = (c, N, e * N + 17 * c, 0.1 * e, np.float32(2 * np.pi * s.doppler_hz / fs), 0.0, 0.0,
                               np.float32(1.023e6 / fs), 0.0)
    dev = torch.from_numpy(x.view(np.float32)).cuda()
    jdev = torch.from_numpy(jobs.view(np.uint8)).cuda()
    out = torch.zeros(C * E * 3 * 2, dtype=torch.float32, device="cuda")
    corr.run_epochs(jdev.data_ptr(), C, E, dev.data_ptr(), len(x), out.data_ptr())
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.complex64).reshape(E * C, 3)
    for i, j in enumerate(jobs):
        seg = x[j["sample_offset"]:j["sample_offset"] + N]
        ref = volk.multicorrelator_real_codes_exact(seg, synth.gps_ca_chips(sats[j["channel"]].prn), shifts,
                                                    float(j["rem_carr_phase_rad"]), float(j["carr_phase_step_rad"]),
                                                    0.0, float(j["code_phase_step_chips"]), N)
        assert vnorm_rel(o[i], ref) <= 2e-5
