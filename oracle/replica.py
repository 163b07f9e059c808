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
