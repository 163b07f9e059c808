"""Seeded synthetic GNSS IQ generator used by tests and bench.py.

IQ = sum_p A_p * code_p(t - tau_p) * b_p(t) * exp(j(2*pi*f_p*t + theta_p)) + AWGN
with complex noise variance 1 and A_p = sqrt(10^(CN0/10) / fs).  Identical inputs
for the CPU baseline and the GPU (numpy PCG64 seeded with 0x5EED + config id).

The GPS L1 C/A chips come from the engine's own code generator restated here
(G1/G2 LFSR, IS-GPS-200) so this module has no dependency on oracle/.
"""
import numpy as np

SEED = 0x5EED

_G2_DELAYS = [5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469, 470,
              471, 472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862]


def _lfsr(taps):
    reg = [1] * 10
    out = np.zeros(1023, np.int8)
    for i in range(1023):
        out[i] = reg[0]
        fb = 0
        for t in taps:
            fb ^= reg[t]
        reg = reg[1:] + [fb]
    return out


_G1 = _lfsr([7, 0])
_G2 = _lfsr([8, 7, 4, 2, 1, 0])


def gps_ca_chips(prn):
    """+-1 chips of GPS L1 C/A PRN 1..32 (logic 1 -> +1)."""
    d = (1023 - _G2_DELAYS[prn - 1]) % 1023
    bits = _G1 ^ _G2[(d + np.arange(1023)) % 1023]
    return np.where(bits == 1, 1.0, -1.0).astype(np.float32)


def gps_ca_sampled(prn, fs, n=None):
    """Acquisition replica sampled at fs (complex (0, +-1)), as in
    gps_l1_ca_code_gen_complex_sampled (float32 index arithmetic)."""
    f32 = np.float32
    spc = int(float(fs) / (1023000.0 / 1023.0))
    tc = f32(1.0) / f32(1023000)
    ts = f32(1.0) / f32(fs)
    i = np.arange(spc, dtype=np.float32)
    idx = (((ts * (i + f32(1))) / tc) + f32(1)).astype(np.int64).astype(np.int32) - 1
    idx[-1] = 1022
    c = np.zeros(spc, np.complex64)
    c.imag = gps_ca_chips(prn)[idx]
    if n is not None and n != spc:
        c = np.resize(c, n)
    return c


GPS_L1_HZ = 1.57542e9
GPS_PREAMBLE = (1, 0, 0, 0, 1, 0, 1, 1)  # TLM preamble 10001011 (GPS_L1_CA.h:61-73)


class Satellite:
    """preamble_every_bits: when set, the navigation bit stream carries the GPS TLM
    preamble every that many bits (bit synchronisation in tracking needs it);
    code_doppler: the code rate follows the carrier Doppler (1 + f_d / f_L1)."""

    def __init__(self, prn, doppler_hz, code_delay_chips, cn0_dbhz=45.0, phase=0.0, bit_period_ms=20,
                 preamble_every_bits=None, code_doppler=False):
        self.prn = prn
        self.doppler_hz = doppler_hz
        self.code_delay_chips = code_delay_chips
        self.cn0_dbhz = cn0_dbhz
        self.phase = phase
        self.bit_period_ms = bit_period_ms
        self.preamble_every_bits = preamble_every_bits
        self.code_doppler = code_doppler

    def nav_bits(self, nbits):
        bits_rng = np.random.default_rng(SEED + 77 * self.prn)
        bits = np.where(bits_rng.random(nbits) < 0.5, -1.0, 1.0)
        if self.preamble_every_bits:
            pre = np.array([1.0 if b else -1.0 for b in GPS_PREAMBLE])
            for k in range(0, nbits - len(pre) + 1, self.preamble_every_bits):
                bits[k:k + len(pre)] = pre
        return bits


def random_constellation(n_visible=8, seed_offset=0, cn0_dbhz=45.0, max_doppler=9000.0, prns=None):
    rng = np.random.default_rng(SEED + seed_offset)
    if prns is None:
        prns = sorted(rng.choice(np.arange(1, 33), size=n_visible, replace=False).tolist())
    sats = []
    for p in prns:
        sats.append(Satellite(int(p), float(rng.uniform(-max_doppler, max_doppler)), float(rng.uniform(0, 1023)),
                              cn0_dbhz, float(rng.uniform(0, 2 * np.pi))))
    return sats


def gps_l1_iq(fs, n_samples, sats, seed_offset=0, t0_samples=0, noise=True, dtype=np.complex64):
    """Generate n_samples of complex64 IQ at fs starting at sample t0_samples."""
    rng = np.random.default_rng(SEED + 1000 + seed_offset + t0_samples)
    t = (np.arange(n_samples, dtype=np.float64) + t0_samples) / fs
    out = np.zeros(n_samples, np.complex128)
    for s in sats:
        chips = gps_ca_chips(s.prn)
        amp = np.sqrt(10.0 ** (s.cn0_dbhz / 10.0) / fs)
        rate = 1.023e6 * (1.0 + s.doppler_hz / GPS_L1_HZ) if s.code_doppler else 1.023e6
        code_phase = t * rate - s.code_delay_chips
        c = chips[np.floor(code_phase).astype(np.int64) % 1023]
        nbits = int(np.ceil((t[-1] + 1) * 1000 / s.bit_period_ms)) + 2
        bits = s.nav_bits(nbits)
        # bit edges follow the code epochs (20 code periods per bit)
        b = bits[np.floor(code_phase / 1023.0 / s.bit_period_ms).astype(np.int64) % nbits]
        out += amp * c * b * np.exp(1j * (2 * np.pi * s.doppler_hz * t + s.phase))
    if noise:
        out += (rng.standard_normal(n_samples) + 1j * rng.standard_normal(n_samples)) * np.sqrt(0.5)
    return out.astype(dtype)


def to_cshort(iq, scale=1000.0):
    """complex -> interleaved int16 (lv_16sc_t), saturating."""
    a = np.empty(2 * len(iq), np.float64)
    a[0::2] = iq.real * scale
    a[1::2] = iq.imag * scale
    return np.clip(np.rint(a), -32768, 32767).astype(np.int16)
