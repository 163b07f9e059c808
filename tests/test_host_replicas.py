"""C++ replica generators of the host adapters (gnss-sdr-new_amd/host/gnss_replicas.cc)
against the oracle restatement (oracle/replica.py), bit-exact, no GPU:
GPS L1 C/A (gps_sdr_signal_replica.cc:25-176), Galileo E1 B/C sinBOC(1,1) and CBOC
(galileo_e1_signal_replica.cc:29-233, ICD memory codes), BeiDou B1I
(beidou_b1i_signal_replica.cc:26-176)."""
import os
import subprocess

import numpy as np
import pytest

from oracle import replica

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "gnss-sdr-new_amd", "build", "replica_dump")


def dump(*args, dtype=np.float32):
    if not os.path.exists(TOOL):
        pytest.skip("replica_dump not built (python __graft_entry__.py)")
    out = subprocess.run([TOOL] + [str(a) for a in args], check=True, capture_output=True).stdout
    v = np.frombuffer(out, np.float32)
    return v.view(np.complex64) if dtype == np.complex64 else v


@pytest.mark.parametrize("prn", [1, 7, 19, 32])
def test_gps(prn):
    np.testing.assert_array_equal(dump("gps_float", prn), replica.gps_l1_ca_code_int(prn).astype(np.float32))
    for fs in (2000000, 4000000, 16000000, 25000000):
        got = dump("gps_sampled", prn, fs, dtype=np.complex64)
        np.testing.assert_array_equal(got, replica.gps_l1_ca_code_complex_sampled(prn, fs))


@pytest.mark.parametrize("prn", [1, 11, 30, 50])
def test_galileo(prn):
    for sig, kind in (("1B", "b"), ("1C", "c")):
        np.testing.assert_array_equal(dump("gal_%s_sinboc11" % kind, prn),
                                      replica.galileo_e1_code_sinboc11_float(sig, prn))
        for fs in (4000000, 8000000, 25000000):
            for cboc in (0, 1):
                got = dump("gal_%s_sampled" % kind, prn, fs, cboc, 0, dtype=np.complex64)
                np.testing.assert_array_equal(got, replica.galileo_e1_code_complex_sampled(sig, bool(cboc), prn, fs))
    got = dump("gal_c_sampled", prn, 4000000, 0, 1, dtype=np.complex64)
    np.testing.assert_array_equal(got, replica.galileo_e1_code_complex_sampled("1C", False, prn, 4000000, secondary=True))


@pytest.mark.parametrize("prn", [1, 6, 37, 38, 53, 54, 57, 63])
def test_beidou(prn):
    np.testing.assert_array_equal(dump("bds_float", prn), replica.beidou_b1i_code_float(prn))
    for fs in (4000000, 25000000):
        np.testing.assert_array_equal(dump("bds_sampled", prn, fs, dtype=np.complex64),
                                      replica.beidou_b1i_code_complex_sampled(prn, fs))
