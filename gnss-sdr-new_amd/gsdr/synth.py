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
                 preamble_every_bits=None, code_doppler=False, doppler_rate_hz_s=0.0):
        self.prn = prn
        self.doppler_rate_hz_s = doppler_rate_hz_s  # linear Doppler ramp (high-dynamics tests)
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
        ramp = getattr(s, "doppler_rate_hz_s", 0.0)
        if ramp:
            cycles = s.doppler_hz * t + 0.5 * ramp * t * t
            code_phase = t * 1.023e6 + (1.023e6 / GPS_L1_HZ * cycles if s.code_doppler else 0.0) - s.code_delay_chips
        else:
            cycles = None
            code_phase = t * rate - s.code_delay_chips
        c = chips[np.floor(code_phase).astype(np.int64) % 1023]
        nbits = int(np.ceil((t[-1] + 1) * 1000 / s.bit_period_ms)) + 2
        bits = s.nav_bits(nbits)
        # bit edges follow the code epochs (20 code periods per bit)
        b = bits[np.floor(code_phase / 1023.0 / s.bit_period_ms).astype(np.int64) % nbits]
        if cycles is not None:
            out += amp * c * b * np.exp(1j * (2 * np.pi * cycles + s.phase))
        else:
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


def to_ibyte(iq, scale=20.0):
    """complex -> interleaved int8 I,Q (SignalSource.item_type=byte), saturating."""
    a = np.empty(2 * len(iq), np.float64)
    a[0::2] = iq.real * scale
    a[1::2] = iq.imag * scale
    return np.clip(np.rint(a), -128, 127).astype(np.int8)


def ibyte_to_complex(b):
    """Ibyte_To_Complex (gr::blocks::interleaved_char_to_complex, scale 1)."""
    b = np.asarray(b, np.int8).astype(np.float32)
    return (b[0::2] + 1j * b[1::2]).astype(np.complex64)


# ---------------------------------------------------------------- Galileo E1, BeiDou B1I
# Code tables: Galileo OS SIS ICD memory codes (data/galileo_e1_codes.bin, see
# tools/extract_galileo_e1_codes.py); BeiDou B1I Gold codes from the ICD's G1/G2
# registers and phase assignment.
import os as _os

GAL_E1_HZ = 1.57542e9
BDS_B1I_HZ = 1.561098e9
_GAL_TABLE = None
GAL_E1C_SECONDARY = "0011100000001010110110010"
BDS_B1I_NH = "00000100110101001110"


def gal_e1_chips(prn, pilot=False):
    """+-1 chips (logic 0 -> +1) of E1-B (data) or E1-C (pilot) PRN 1..50."""
    global _GAL_TABLE
    if _GAL_TABLE is None:
        path = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "data", "galileo_e1_codes.bin")
        _GAL_TABLE = np.unpackbits(np.fromfile(path, np.uint8).reshape(100, 512), axis=1)[:, :4092]
    return (1.0 - 2.0 * _GAL_TABLE[(50 if pilot else 0) + prn - 1]).astype(np.float32)


def gal_e1_sinboc11(prn, pilot=False):
    """Tracking replica: sinBOC(1,1) at 2 samples per chip (+c, -c) -- 8184 floats."""
    c = gal_e1_chips(prn, pilot)
    return np.stack([c, -c], axis=1).reshape(-1)


def _f32_upsample_index(n, fs_in, fs_out):
    """idx = (int)(t_out*(i+1)*fs_in + 1) - 1 in float32, last one forced (the
    reference replica samplers' index rule)."""
    f32 = np.float32
    i = np.arange(n, dtype=np.float32)
    idx = (((f32(1.0) / f32(fs_out)) * (i + f32(1.0))) * f32(fs_in) + f32(1)).astype(np.int64).astype(np.int32) - 1
    return idx


def gal_e1_sampled(prn, fs, pilot=False, cboc=False):
    """Acquisition replica at fs (complex, real part), one 4 ms code period: the
    sinBOC(1,1) (or CBOC(6,1,1/11) at 12 samples/chip) chip stream resampled to fs."""
    c = gal_e1_chips(prn, pilot)
    if cboc:
        a = np.float32(np.sqrt(np.float32(10.0) / np.float32(11.0)))
        b = np.float32(np.sqrt(np.float32(1.0) / np.float32(11.0)))
        s11 = np.repeat(np.array([1.0] * 6 + [-1.0] * 6, np.float32)[None, :], 4092, 0) * c[:, None]
        s61 = np.repeat(np.array([1.0, -1.0] * 6, np.float32)[None, :], 4092, 0) * c[:, None]
        sub = (a * s11 + b * s61) if not pilot else (a * s11 - b * s61)
        src, rate = sub.reshape(-1).astype(np.float32), 12 * 1023000
    else:
        src, rate = gal_e1_sinboc11(prn, pilot), 2 * 1023000
    n = int(float(fs) / (1023000.0 / 4092.0))
    if fs != rate:
        idx = _f32_upsample_index(n, float(rate), fs)
        idx[-1] = len(src) - 1
        src = src[idx]
    return src.astype(np.complex64)


def _bds_registers():
    init = [int("01010101010"[10 - i]) for i in range(11)]
    return list(init), list(init)


def bds_b1i_chips(prn):
    """+-1 chips of BeiDou B1I PRN 1..63 (G1 xor phase-selected G2 taps; logic 1 -> +1)."""
    ph = {1: (1, 3), 2: (1, 4), 3: (1, 5), 4: (1, 6), 5: (1, 8), 6: (1, 9), 7: (1, 10), 8: (1, 11), 9: (2, 7),
          10: (3, 4), 11: (3, 5), 12: (3, 6), 13: (3, 8), 14: (3, 9), 15: (3, 10), 16: (3, 11), 17: (4, 5),
          18: (4, 6), 19: (4, 8), 20: (4, 9), 21: (4, 10), 22: (4, 11), 23: (5, 6), 24: (5, 8), 25: (5, 9),
          26: (5, 10), 27: (5, 11), 28: (6, 8), 29: (6, 9), 30: (6, 10), 31: (6, 11), 32: (8, 9), 33: (8, 10),
          34: (8, 11), 35: (9, 10), 36: (9, 11), 37: (10, 11)}
    ph3 = {38: (1, 2, 7), 39: (1, 3, 4), 40: (1, 3, 6), 41: (1, 3, 8), 42: (1, 3, 10), 43: (1, 3, 11),
           44: (1, 4, 5), 45: (1, 4, 9), 46: (1, 5, 6), 47: (1, 5, 8), 48: (1, 5, 10), 49: (1, 5, 11), 50: (1, 6, 9),
           51: (1, 8, 9), 52: (1, 9, 10), 53: (1, 9, 11), 54: (2, 3, 7), 55: (2, 5, 7), 56: (2, 7, 9),
           57: (3, 4, 5), 58: (3, 4, 9), 59: (3, 5, 6), 60: (3, 5, 8), 61: (3, 5, 10), 62: (3, 5, 11),
           63: (3, 6, 9)}
    taps = ph[prn] if prn in ph else ph3[prn]
    g1r, g2r = _bds_registers()
    g1 = np.zeros(2046, np.int8)
    g2 = np.zeros(2046, np.int8)
    for i in range(2046):
        g1[i] = g1r[0]
        v = 0
        for t in taps:
            v ^= g2r[11 - t]
        g2[i] = v
        f1 = g1r[0] ^ g1r[1] ^ g1r[2] ^ g1r[3] ^ g1r[4] ^ g1r[10]
        f2 = g2r[0] ^ g2r[2] ^ g2r[3] ^ g2r[6] ^ g2r[7] ^ g2r[8] ^ g2r[9] ^ g2r[10]
        g1r = g1r[1:] + [f1]
        g2r = g2r[1:] + [f2]
    return np.where((g1 ^ g2) == 1, 1.0, -1.0).astype(np.float32)


def bds_b1i_sampled(prn, fs):
    """Acquisition replica at fs (complex, real +-1), one 1 ms code period."""
    n = int(float(fs) / (2046000.0 / 2046.0))
    f32 = np.float32
    i = np.arange(n, dtype=np.float32)
    idx = ((((f32(1.0) / f32(fs)) * (i + f32(1))) / (f32(1.0) / f32(2046000))) + f32(1)).astype(np.int64).astype(np.int32) - 1
    idx[-1] = 2045
    return bds_b1i_chips(prn)[idx].astype(np.complex64)


class GalileoSatellite:
    """E1 OS signal: (E1-B data - E1-C pilot x secondary) / sqrt(2), CBOC(6,1,1/11)
    subcarriers, 4 ms symbols on E1-B."""

    def __init__(self, prn, doppler_hz, code_delay_chips, cn0_dbhz=45.0, phase=0.0):
        self.prn, self.doppler_hz, self.code_delay_chips = prn, doppler_hz, code_delay_chips
        self.cn0_dbhz, self.phase = cn0_dbhz, phase


def gal_e1_iq(fs, n_samples, sats, seed_offset=0, noise=True, dtype=np.complex64):
    rng = np.random.default_rng(SEED + 2000 + seed_offset)
    t = np.arange(n_samples, dtype=np.float64) / fs
    out = np.zeros(n_samples, np.complex128)
    a, b = np.sqrt(10.0 / 11.0), np.sqrt(1.0 / 11.0)
    sec = np.array([1.0 if c == "0" else -1.0 for c in GAL_E1C_SECONDARY])
    for s in sats:
        amp = np.sqrt(10.0 ** (s.cn0_dbhz / 10.0) / fs)
        # the code rate follows the carrier Doppler (1 + f_d / f_E1)
        cp = t * 1.023e6 * (1.0 + s.doppler_hz / GAL_E1_HZ) - s.code_delay_chips  # chips
        chip = np.floor(cp).astype(np.int64)
        frac = cp - chip
        s11 = np.where(frac < 0.5, 1.0, -1.0)
        s61 = np.where(np.floor(frac * 12).astype(np.int64) % 2 == 0, 1.0, -1.0)
        epoch = np.floor_divide(chip, 4092)
        cb = gal_e1_chips(s.prn)[chip % 4092]
        cc = gal_e1_chips(s.prn, pilot=True)[chip % 4092]
        brng = np.random.default_rng(SEED + 91 * s.prn)
        nb = int(epoch.max() - epoch.min()) + 2
        bits = np.where(brng.random(nb) < 0.5, -1.0, 1.0)
        d = bits[(epoch - epoch.min()) % nb]
        e1b = cb * d * (a * s11 + b * s61)
        e1c = cc * sec[epoch % 25] * (a * s11 - b * s61)
        out += amp * (e1b - e1c) / np.sqrt(2.0) * np.exp(1j * (2 * np.pi * s.doppler_hz * t + s.phase))
    if noise:
        out += (rng.standard_normal(n_samples) + 1j * rng.standard_normal(n_samples)) * np.sqrt(0.5)
    return out.astype(dtype)


BDS_D2_PREAMBLE_BITS = (1, 1, 1, 0, 0, 0, 1, 0, 0, 1, 0)  # BEIDOU_B1I_GEO_PREAMBLE_SYMBOLS_STR, 2 symbols/bit


def bds_is_geo(prn):
    return 0 < prn < 6 or prn > 58


def bds_b1i_iq(fs, n_samples, sats, seed_offset=0, noise=True, dtype=np.complex64, code_doppler=True):
    """B1I signal; sats are Satellite objects whose code_delay_chips is in B1I chips
    (2.046 Mcps).  MEO/IGSO (D1): code x NH(20) x 50 bps data.  GEO (PRN 1-5,
    59-63, D2): code x 500 bps data (2 code periods per bit) carrying the D2
    preamble every 300 bits.  code_doppler=False keeps the chip rate at 2.046 Mcps
    (a span repeated end to end is then continuous in code phase)."""
    rng = np.random.default_rng(SEED + 3000 + seed_offset)
    t = np.arange(n_samples, dtype=np.float64) / fs
    out = np.zeros(n_samples, np.complex128)
    nh = np.array([1.0 if c == "0" else -1.0 for c in BDS_B1I_NH])
    for s in sats:
        amp = np.sqrt(10.0 ** (s.cn0_dbhz / 10.0) / fs)
        cp = t * 2.046e6 * ((1.0 + s.doppler_hz / BDS_B1I_HZ) if code_doppler else 1.0) - s.code_delay_chips
        chip = np.floor(cp).astype(np.int64)
        epoch = np.floor_divide(chip, 2046)
        c = bds_b1i_chips(s.prn)[chip % 2046]
        geo = bds_is_geo(s.prn)
        per = 2 if geo else 20
        bit = np.floor_divide(epoch, per)
        nb = int(bit.max() - bit.min()) + 2
        bits = np.where(np.random.default_rng(SEED + 53 * s.prn).random(nb) < 0.5, -1.0, 1.0)
        if geo:
            pre = np.array([1.0 if b else -1.0 for b in BDS_D2_PREAMBLE_BITS])
            for k in range(0, nb - len(pre) + 1, 300):
                bits[k:k + len(pre)] = pre
            mod = np.ones_like(cp)
        else:
            mod = nh[epoch % 20]
        out += amp * c * mod * bits[(bit - bit.min()) % nb] * np.exp(1j * (2 * np.pi * s.doppler_hz * t + s.phase))
    if noise:
        out += (rng.standard_normal(n_samples) + 1j * rng.standard_normal(n_samples)) * np.sqrt(0.5)
    return out.astype(dtype)
