"""ORACLE — test infrastructure only.

Restatement of GNSS-SDR's Parallel Code Phase Search acquisition core
(src/algorithms/acquisition/gnuradio_blocks/pcps_acquisition.cc) with numpy.
The FFT library boundary (FFTW3f through gr-fft in the reference) is restated
with numpy's pocketfft: in complex128 ("exact", default) or complex64.  Both
directions are unnormalised like FFTW (gnss_sdr_fft.h:22-63).

Pinned by the reference's own acquisition validation tests on its IQ captures
(tests/test_oracle_golden.py: GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat, delay 524 samples
/ Doppler 1680 Hz within the reference's 0.5 chip / 666 Hz tolerances).
"""
import math

import numpy as np
from scipy.special import gammaincinv

from . import volk

TWO_PI = 6.283185307179586


def num_doppler_bins(doppler_max, doppler_step):
    """pcps_acquisition.cc:264 — ceil((dmax - (-dmax)) / step)."""
    return int(math.ceil(float(int(doppler_max) - int(-doppler_max)) / float(doppler_step)))


def doppler_hz(d, doppler_max, doppler_step, doppler_center=0):
    """pcps_acquisition.cc:302 and :537."""
    return -int(doppler_max) + int(doppler_center) + int(doppler_step) * int(d)


# Carrier wipe-off models (GNSS-SDR computes the carrier with the VOLK protokernel
# volk_gnsssdr_s32f_sincos_32fc that its dispatcher selects for the host):
#   "exact"   exp(-j 2 pi f n / fs) evaluated in fp64 and rounded once -- the MI355X
#             engine's default (gsdr_acq_set_wipeoff, GSDR_WIPE_EXACT);
#   "generic" the generic protokernel (KERN/s32f_sincos_32fc.h:390-403): one fp32
#             phase accumulator, cosf / sinf;
#   "avx2"    the a_avx2 / u_avx2 protokernel (:448-627) an AVX2 x86-64 host runs:
#             eight fp32 accumulators advancing by 8 inc, Cephes polynomials.
# The two protokernels' accumulated fp32 phase drifts from the exact carrier (C2:
# 1e-3 / 2e-5 rad, C4 64000 points: 0.15 / 0.01 rad); DESIGN.md 3 states the bar.
WIPE_MODES = ("exact", "generic", "avx2")


def carrier(freq, fs, N, mode="exact"):
    """One wipe-off row for the float frequency freq (update_local_carrier, :233-246)."""
    f32 = np.float32
    f = f32(freq)
    if mode == "exact":
        t = float(f) * np.arange(N, dtype=np.float64) / float(fs)
        return np.exp(-2j * np.pi * (t - np.floor(t))).astype(np.complex64)
    step = f32(TWO_PI) * f / f32(fs)
    if mode == "generic":
        return volk.s32f_sincos_32fc(float(-step), N)
    if mode == "avx2":
        return volk.s32f_sincos_32fc_avx2(float(-step), N)
    raise ValueError(mode)


def doppler_wipeoffs(fs, N, doppler_max, doppler_step, D, doppler_center=0, doppler_bias=0, mode="exact"):
    """update_grid_doppler_wipeoffs (:298-305) + update_local_carrier (:233-246):
    phase_step = float(TWO_PI) * f / float(fs) in float32 and -phase_step through the
    sincos model `mode` (see carrier)."""
    w = np.empty((D, N), np.complex64)
    for d in range(D):
        f = np.float32(doppler_bias + doppler_hz(d, doppler_max, doppler_step, doppler_center))
        w[d] = carrier(f, fs, N, mode)
    return w


def fft_code(code, fft_size, consumed, bit_transition=False, dtype=np.complex128):
    """set_local_code (:176-209): place code in the FFT buffer, FFT, conjugate."""
    buf = np.zeros(fft_size, dtype)
    if bit_transition:
        off = fft_size // 2
        buf[off:] = code[:off]
    elif fft_size == consumed:
        buf[:] = code[:consumed]
    else:
        buf[fft_size - consumed:] = code[:consumed]
    return np.conj(np.fft.fft(buf)).astype(dtype)


def magnitude_grid(x, wipe, code_fft, bit_transition=False, dtype=np.complex128):
    """The Doppler loop of acquisition_core (:655-686): |IFFT(FFT(x*w_d) . Cconj)|^2,
    unnormalised inverse (FFTW rev = N * numpy.ifft).  Returns float32 [D][Neff]."""
    D, N = wipe.shape
    xs = x.astype(dtype)
    t = xs[None, :] * wipe.astype(dtype)
    if dtype == np.complex64:
        t = t.astype(np.complex64)
    X = np.fft.fft(t, axis=1)
    R = np.fft.ifft(X * code_fft[None, :].astype(dtype), axis=1) * N
    M = (R.real.astype(np.float64) ** 2 + R.imag.astype(np.float64) ** 2)
    if bit_transition:
        M = M[:, N // 2:]
    return M.astype(np.float32)


def magnitude_grids(x, wipe, code_ffts, bit_transition=False):
    """magnitude_grid for several PRNs over one block: the Doppler rows' forward
    transforms X_d = FFT(x . w_d) (:655-662) do not depend on the PRN, so they are
    computed once and every PRN's grid is |IFFT(X . C_p)|^2 (:663-666) -- the same
    arithmetic as magnitude_grid, one PRN at a time (yields float32 [D][Neff])."""
    D, N = wipe.shape
    X = np.fft.fft(x.astype(np.complex128)[None, :] * wipe.astype(np.complex128), axis=1)
    for cf in code_ffts:
        R = np.fft.ifft(X * cf[None, :].astype(np.complex128), axis=1) * N
        M = R.real ** 2 + R.imag ** 2
        if bit_transition:
            M = M[:, N // 2:]
        yield M.astype(np.float32)


def max_to_input_power_statistic(M, dwells=1):
    """pcps_acquisition.cc:511-543 (first-step branch).  Returns
    (index_time, index_doppler, grid_max, input_power, statistic)."""
    D, Neff = M.shape
    gmax = np.float32(0.0)
    di = 0
    ti = 0
    for i in range(D):
        t = volk.index_max_32u(M[i])
        if M[i, t] > gmax:
            gmax = M[i, t]
            di = i
            ti = t
    opp = (di + D // 2) % D
    acc = np.float32(0.0)
    # std::accumulate in float; vectorised sequential sum via cumsum (strictly ordered)
    acc = np.cumsum(M[opp], dtype=np.float32)[-1]
    # float accumulate / int32 is a float division; then / 2.0 / counter in double (:533)
    input_power = np.float32(float(np.float32(acc) / np.float32(Neff)) / 2.0 / dwells)
    return ti, di, np.float32(gmax), input_power, np.float32(gmax / input_power)


def first_vs_second_peak_statistic(M, samples_per_chip, fft_size):
    """pcps_acquisition.cc:546-612, including its one-sided wrap of the exclusion
    window.  Returns (index_time, index_doppler, first, second, statistic)."""
    D, _ = M.shape
    first = np.float32(0.0)
    di = 0
    ti = 0
    for i in range(D):
        t = volk.index_max_32u(M[i])
        if M[i, t] > first:
            first = M[i, t]
            di = i
            ti = t
    e1 = ti - samples_per_chip
    e2 = ti + samples_per_chip
    if e1 < 0:
        e1 = fft_size + e1
    elif e2 >= fft_size:
        e2 = e2 - fft_size
    tmp = M[di].copy()
    idx = e1
    while True:
        tmp[idx] = 0.0
        idx += 1
        if idx == fft_size:
            idx = 0
        if idx == e2:
            break
    second = tmp[volk.index_max_32u(tmp)]
    return ti, di, np.float32(first), np.float32(second), np.float32(first / second)


def threshold(pfa, fft_size, D, max_dwells=1, bit_transition=False):
    """calculate_threshold (:894-909) with Boost gamma_p_inv == scipy gammaincinv."""
    if pfa <= 0.0:
        return None
    neff = fft_size // 2 if bit_transition else fft_size
    nb = neff * D
    a = 2.0 * (1 if bit_transition else max_dwells)
    p = math.pow(1.0 - float(np.float32(pfa)), 1.0 / float(np.float32(nb)))
    return float(np.float32(2.0 * gammaincinv(a, p)))


class AcqResult:
    __slots__ = ("index_time", "index_doppler", "doppler_hz", "peak", "input_power", "second_peak",
                 "test_statistic", "delay_samples")

    def __repr__(self):
        return "AcqResult(t=%d, d=%d, dop=%d, peak=%g, stat=%g)" % (
            self.index_time, self.index_doppler, self.doppler_hz, self.peak, self.test_statistic)


def acquire(x, code, fs, doppler_max, doppler_step, D=None, pfa=0.0, samples_per_chip=None,
            samples_per_code=None, doppler_center=0, dwells=1, dtype=np.complex128, wipe=None, M_out=None):
    """One acquisition_core pass (single dwell, no bit transition) for one PRN.
    x, code: complex64[N].  Returns AcqResult."""
    N = len(x)
    if D is None:
        D = num_doppler_bins(doppler_max, doppler_step)
    if wipe is None:
        wipe = doppler_wipeoffs(fs, N, doppler_max, doppler_step, D, doppler_center)
    cf = fft_code(code, N, N, dtype=dtype)
    M = magnitude_grid(x, wipe, cf, dtype=dtype)
    if M_out is not None:
        M_out.append(M)
    r = AcqResult()
    if samples_per_chip is None:
        samples_per_chip = int(math.ceil(float(np.float32(fs)) / 1023000.0))
    if samples_per_code is None:
        samples_per_code = float(np.float32(np.float32(fs) * np.float32(0.001)))
    if pfa > 0.0:
        ti, di, gmax, ip, stat = max_to_input_power_statistic(M, dwells)
        r.peak, r.input_power, r.second_peak = gmax, ip, np.float32(0)
    else:
        ti, di, first, second, stat = first_vs_second_peak_statistic(M, samples_per_chip, N)
        r.peak, r.input_power, r.second_peak = first, np.float32(0), second
    r.index_time, r.index_doppler, r.test_statistic = int(ti), int(di), stat
    r.doppler_hz = doppler_hz(di, doppler_max, doppler_step, doppler_center)
    r.delay_samples = float(np.fmod(np.float32(ti), np.float32(samples_per_code)))
    return r


# ---------------------------------------------------------------- make_two_steps
def step_two_freqs(center2, doppler_step2, nbins2):
    """update_grid_doppler_wipeoffs_step2 (:307-314): float32
    (float(d) - float(floor(nbins2 / 2.0))) * step2, then + centre."""
    f32 = np.float32
    half = f32(math.floor(nbins2 / 2.0))
    return [f32(f32(center2) + f32(f32(f32(d) - half) * f32(doppler_step2))) for d in range(nbins2)]


def doppler_wipeoffs_step2(fs, N, center2, doppler_step2, nbins2, mode="exact"):
    """The narrow grid's carriers (update_local_carrier with float freq, :233-246)."""
    w = np.empty((nbins2, N), np.complex64)
    for d, f in enumerate(step_two_freqs(center2, doppler_step2, nbins2)):
        w[d] = carrier(np.float32(f), fs, N, mode)
    return w


def step_two_doppler_hz(d, center2, doppler_step2, nbins2):
    """:539 / :576 — static_cast<int32_t>(centre + (float(d) - float(floor(n/2.0))) * step2)."""
    f32 = np.float32
    v = f32(f32(center2) + f32(f32(f32(d) - f32(math.floor(nbins2 / 2.0))) * f32(doppler_step2)))
    return int(np.trunc(v))


def step_two_statistic(M, coarse_input_power, center2, doppler_step2, samples_per_chip=None, fft_size=None,
                       cfar=True):
    """The step-two branch of acquisition_core (:744-773): CFAR divides the narrow-grid
    maximum by the FIRST step's d_input_power (the step-two branch of
    max_to_input_power_statistic does not recompute it, :530-540); the peak ratio is
    unchanged.  Returns (index_time, index_doppler, peak, second_peak, statistic, doppler_hz)."""
    nb = M.shape[0]
    if cfar:
        D, _ = M.shape
        gmax = np.float32(0.0)
        di = ti = 0
        for i in range(D):
            t = volk.index_max_32u(M[i])
            if M[i, t] > gmax:
                gmax, di, ti = M[i, t], i, t
        stat = np.float32(np.float32(gmax) / np.float32(coarse_input_power))
        second = np.float32(0)
    else:
        ti, di, gmax, second, stat = first_vs_second_peak_statistic(M, samples_per_chip, fft_size)
    return int(ti), int(di), np.float32(gmax), second, stat, step_two_doppler_hz(di, center2, doppler_step2, nb)


def threshold_step_two(pfa, pfa2, fft_size, nbins2, max_dwells=1, bit_transition=False, first_threshold=None):
    """calculate_threshold with d_step_two (:894-909); pfa2 outside (0,1] is pfa
    (acq_conf.cc:72-76); pfa2 <= 0 keeps the first-step threshold."""
    if pfa2 <= 0.0 or pfa2 > 1.0:
        pfa2 = pfa
    if pfa2 <= 0.0:
        return first_threshold
    return threshold(pfa2, fft_size, nbins2, max_dwells, bit_transition)
