"""ORACLE — test infrastructure only.

Restatement of the GNSS-SDR code replica generators used on the acquisition and
tracking hot path.  Used by tests/ (and bench.py's cpu_baseline leg) as the
checker for the product's own C++ replica code (gnss-sdr-new_amd/host/).

Pinned by the IS-GPS-200 "first 10 chips (octal)" known-answer table for PRN
1-32 (tests/test_oracle_golden.py) and by reproducing the reference's own
acquisition golden results on the reference's captures.
"""
import numpy as np

# G2 delays, src/algorithms/libs/gps_sdr_signal_replica.cc:42-45 (PRN 1-32, SBAS 120-138)
_G2_DELAYS = [5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469, 470,
              471, 472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862,
              145, 175, 52, 21, 237, 235, 886, 657, 634, 762, 355, 1012, 176, 603, 130, 359,
              595, 68, 386]

GPS_L1_CA_CODE_LENGTH_CHIPS = 1023
GPS_L1_CA_CODE_RATE_CPS = 1.023e6


def _gold_registers():
    """G1/G2 output sequences, gps_sdr_signal_replica.cc:64-80."""
    g1r = [1] * 10
    g2r = [1] * 10
    g1 = np.zeros(1023, np.int8)
    g2 = np.zeros(1023, np.int8)
    for i in range(1023):
        g1[i] = g1r[0]
        g2[i] = g2r[0]
        f1 = g1r[7] ^ g1r[0]
        f2 = g2r[8] ^ g2r[7] ^ g2r[4] ^ g2r[2] ^ g2r[1] ^ g2r[0]
        g1r = g1r[1:] + [f1]
        g2r = g2r[1:] + [f2]
    return g1, g2


_G1, _G2 = _gold_registers()


def gps_l1_ca_code_int(prn, chip_shift=0):
    """gps_l1_ca_code_gen_int, gps_sdr_signal_replica.cc:25-102: +1 where G1^G2 is 1."""
    idx = prn - 88 if 120 <= prn <= 138 else prn - 1
    if idx < 0 or idx > 50:
        raise ValueError("unsupported PRN %d" % prn)
    L = 1023
    delay = (L - _G2_DELAYS[idx] + chip_shift) % L
    lcv = np.arange(L)
    bits = _G1[(lcv + chip_shift) % L] ^ _G2[(delay + lcv) % L]
    return np.where(bits == 1, 1, -1).astype(np.int32)


def gps_l1_ca_code_float(prn, chip_shift=0):
    """gps_l1_ca_code_gen_float, gps_sdr_signal_replica.cc:104-115."""
    return gps_l1_ca_code_int(prn, chip_shift).astype(np.float32)


def gps_l1_ca_code_complex(prn, chip_shift=0):
    """gps_l1_ca_code_gen_complex, gps_sdr_signal_replica.cc:118-131: value is (0, +-1)."""
    c = np.zeros(1023, np.complex64)
    c.imag = gps_l1_ca_code_int(prn, chip_shift)
    return c


def gps_l1_ca_code_complex_sampled(prn, fs, chip_shift=0):
    """gps_l1_ca_code_gen_complex_sampled, gps_sdr_signal_replica.cc:136-176.

    Index arithmetic in float32: aux = (ts*(i+1))/tc, idx = (int)(aux+1) - 1,
    last sample forced to the last chip."""
    f32 = np.float32
    code_freq, L = 1023000, 1023
    spc = int(float(fs) / (float(code_freq) / float(L)))
    tc = f32(1.0) / f32(code_freq)
    ts = f32(1.0) / f32(fs)
    chips = gps_l1_ca_code_complex(prn, chip_shift)
    i = np.arange(spc, dtype=np.float32)
    aux = (ts * (i + f32(1))) / tc
    idx = (aux + f32(1)).astype(np.int64).astype(np.int32) - 1
    idx[-1] = L - 1
    return chips[idx]


def first_10_chips_octal(prn):
    """The IS-GPS-200 'first 10 chips' known-answer, as an octal string of the
    logic levels (chip value +1 <-> logic 1 in this generator's convention)."""
    c = gps_l1_ca_code_int(prn)[:10]
    v = 0
    for b in c:
        v = (v << 1) | (1 if b > 0 else 0)
    return "%o" % v


# IS-GPS-200 Table 3-Ia, "First 10 Chips C/A" (octal), PRN 1..32.
IS_GPS_200_FIRST10 = ["1440", "1620", "1710", "1744", "1133", "1455", "1131", "1454", "1626",
                      "1504", "1642", "1750", "1764", "1772", "1775", "1776", "1156", "1467",
                      "1633", "1715", "1746", "1763", "1063", "1706", "1743", "1761", "1770",
                      "1774", "1127", "1453", "1625", "1712"]


# ---------------------------------------------------------------- Galileo E1
# src/algorithms/libs/galileo_e1_signal_replica.cc; code tables from the ICD
# (gnss-sdr-new_amd/gsdr/data/galileo_e1_codes.bin, tools/extract_galileo_e1_codes.py).
GALILEO_E1_CODE_CHIP_RATE_CPS = 1.023e6
GALILEO_E1_B_CODE_LENGTH_CHIPS = 4092
GALILEO_E1_C_SECONDARY_CODE = "0011100000001010110110010"  # Galileo_E1.h:52
_GAL_BIN = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))), "gnss-sdr-new_amd", "gsdr", "data", "galileo_e1_codes.bin")
_GAL = None


def galileo_e1_code_int(signal, prn):
    """galileo_e1_code_gen_int (:29-58) with hex_to_binary_converter
    (gnss_signal_replica.cc:43-...): hex digits MSB first, bit 0 -> +1, bit 1 -> -1."""
    global _GAL
    if _GAL is None:
        raw = np.fromfile(_GAL_BIN, np.uint8).reshape(100, 512)
        _GAL = np.unpackbits(raw, axis=1)[:, :4092]
    if not 1 <= prn <= 50:
        raise ValueError("PRN %d" % prn)
    row = (0 if "1B" in signal else 50) + prn - 1
    return np.where(_GAL[row] == 0, 1, -1).astype(np.int32)


def galileo_e1_sinboc_11_int(prn_chips, length):
    """galileo_e1_sinboc_11_gen_int (:61-77): first half of each chip +c, second half -c."""
    period = length // 4092
    out = np.empty((4092, period), np.int32)
    out[:, :period // 2] = prn_chips[:, None]
    out[:, period // 2:] = -prn_chips[:, None]
    return out.reshape(-1)


def galileo_e1_sinboc_61_int(prn_chips, length):
    """galileo_e1_sinboc_61_gen_int (:80-97): alternating +c, -c."""
    period = length // 4092
    out = np.empty((4092, period), np.int32)
    out[:, 0::2] = prn_chips[:, None]
    out[:, 1::2] = -prn_chips[:, None]
    return out.reshape(-1)


def galileo_e1_code_sinboc11_float(signal, prn):
    """galileo_e1_code_gen_sinboc11_float (:100-111): tracking replica, 2 samples/chip."""
    c = galileo_e1_code_int(signal, prn).astype(np.float32)
    out = np.empty(2 * 4092, np.float32)
    out[0::2] = c
    out[1::2] = -c
    return out


def galileo_e1_gen_float(prn_chips, length, signal):
    """galileo_e1_gen_float (:114-143): CBOC(6,1,1/11), 12 samples/chip, float32."""
    alpha = np.float32(np.sqrt(np.float32(10.0) / np.float32(11.0)))
    beta = np.float32(np.sqrt(np.float32(1.0) / np.float32(11.0)))
    s11 = galileo_e1_sinboc_11_int(prn_chips, length).astype(np.float32)
    s61 = galileo_e1_sinboc_61_int(prn_chips, length).astype(np.float32)
    if "1B" in signal:
        return (alpha * s11 + beta * s61).astype(np.float32)
    return (alpha * s11 - beta * s61).astype(np.float32)


def resampler_float(src, dest_size, fs_in, fs_out):
    """resampler (gnss_signal_replica.cc:257-272): float32 index arithmetic,
    idx = (int)(t_out*(i+1)*fs_in + 1) - 1, last sample forced to the last input."""
    f32 = np.float32
    t_out = f32(1.0) / f32(fs_out)
    i = np.arange(dest_size - 1, dtype=np.float32)
    aux = (t_out * (i + f32(1.0))) * f32(fs_in)
    idx = (aux + f32(1)).astype(np.int64).astype(np.int32) - 1
    out = np.empty(dest_size, src.dtype)
    out[:-1] = src[idx]
    out[-1] = src[-1]
    return out


def galileo_e1_code_float_sampled(signal, cboc, prn, fs, chip_shift=0, secondary=False):
    """galileo_e1_code_gen_float_sampled (:146-210)."""
    code_freq = 1023000
    spc_chip = 12 if cboc else 2
    code_len = spc_chip * 4092
    spcode = int(float(fs) / (float(code_freq) / 4092.0))
    delay = ((4092 - chip_shift) % 4092) * spcode // 4092
    chips = galileo_e1_code_int(signal, prn)
    if cboc:
        sig = galileo_e1_gen_float(chips, code_len, signal)
    else:
        sig = galileo_e1_sinboc_11_int(chips, code_len).astype(np.float32)
    if fs != spc_chip * code_freq:
        sig = resampler_float(sig, spcode, float(spc_chip * code_freq), fs)
    if "1C" in signal and secondary:
        sec = np.array([1.0 if c == "0" else -1.0 for c in GALILEO_E1_C_SECONDARY_CODE], np.float32)
        sig = (sec[:, None] * sig[None, :]).reshape(-1)
        spcode *= 25
    out = np.empty(spcode, np.float32)
    out[(np.arange(spcode) + delay) % spcode] = sig
    return out


def galileo_e1_code_complex_sampled(signal, cboc, prn, fs, chip_shift=0, secondary=False):
    """galileo_e1_code_gen_complex_sampled (:213-233): real part only."""
    return galileo_e1_code_float_sampled(signal, cboc, prn, fs, chip_shift, secondary).astype(np.complex64)


# ---------------------------------------------------------------- BeiDou B1I
# src/algorithms/libs/beidou_b1i_signal_replica.cc
_B1I_PH1 = [1, 1, 1, 1, 1, 1, 1, 1, 2, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 6, 6, 6, 6, 8, 8, 8, 9, 9,
            10, 2, 3, 3, 3, 3, 3, 4, 4, 5, 5, 5, 5, 6, 8, 9, 9, 3, 5, 7, 4, 4, 5, 5, 5, 5, 6]
_B1I_PH2 = [3, 4, 5, 6, 8, 9, 10, 11, 7, 4, 5, 6, 8, 9, 10, 11, 5, 6, 8, 9, 10, 11, 6, 8, 9, 10, 11, 8, 9, 10, 11, 9,
            10, 11, 10, 11, 11, 7, 4, 6, 8, 10, 11, 5, 9, 6, 8, 10, 11, 9, 9, 10, 11, 7, 7, 9, 5, 9, 6, 8, 10, 11, 9]
_B1I_PH3 = [0] * 37 + [1] * 16 + [2] * 3 + [3] * 7
BEIDOU_B1I_SECONDARY_CODE = "00000100110101001110"  # Beidou_B1I.h:44 (NH code)


def beidou_b1i_code_int(prn, chip_shift=0):
    """beidou_b1i_code_gen_int (:26-106).  Registers as std::bitset<11> built from
    "01010101010" (bit i = character 10-i); output G1[0], phase-selected G2 taps
    reg[11-ph]; feedback G1: bits 0,1,2,3,4,10; G2: 0,2,3,6,7,8,9,10."""
    if not 1 <= prn <= 63:
        raise ValueError("PRN %d" % prn)
    L = 2046
    init = "01010101010"
    g1r = [int(init[10 - i]) for i in range(11)]
    g2r = list(g1r)
    p1, p2, p3 = _B1I_PH1[prn - 1], _B1I_PH2[prn - 1], _B1I_PH3[prn - 1]
    g1 = np.zeros(L, np.int8)
    g2 = np.zeros(L, np.int8)
    for i in range(L):
        g1[i] = g1r[0]
        g2[i] = g2r[11 - p1] ^ g2r[11 - p2] ^ (g2r[11 - p3] if p3 else 0)
        f1 = g1r[0] ^ g1r[1] ^ g1r[2] ^ g1r[3] ^ g1r[4] ^ g1r[10]
        f2 = g2r[0] ^ g2r[2] ^ g2r[3] ^ g2r[6] ^ g2r[7] ^ g2r[8] ^ g2r[9] ^ g2r[10]
        g1r = g1r[1:] + [f1]
        g2r = g2r[1:] + [f2]
    lcv = np.arange(L)
    delay = (L + chip_shift) % L
    bits = g1[(lcv + chip_shift) % L] ^ g2[(delay + lcv) % L]
    return np.where(bits == 1, 1, -1).astype(np.int32)


def beidou_b1i_code_float(prn, chip_shift=0):
    """beidou_b1i_code_gen_float (:109-120)."""
    return beidou_b1i_code_int(prn, chip_shift).astype(np.float32)


def beidou_b1i_code_complex_sampled(prn, fs, chip_shift=0):
    """beidou_b1i_code_gen_complex_sampled (:137-176): real +-1, float32 index math."""
    f32 = np.float32
    code_freq, L = 2046000, 2046
    spc = int(float(fs) / (float(code_freq) / float(L)))
    tc = f32(1.0) / f32(code_freq)
    ts = f32(1.0) / f32(fs)
    chips = beidou_b1i_code_int(prn, chip_shift).astype(np.complex64)
    i = np.arange(spc, dtype=np.float32)
    idx = (((ts * (i + f32(1))) / tc) + f32(1)).astype(np.int64).astype(np.int32) - 1
    idx[-1] = L - 1
    return chips[idx]
