import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gnss-sdr-new_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def gps_capture():
    """Reference capture src/tests/signal_samples/GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat (CC-BY-4.0)."""
    return np.fromfile(os.path.join(GOLDEN, "GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat"), np.complex64)


def ccompare(a, b):
    """VOLK-GNSSSDR QA metric (VOLK/lib/qa_utils.cc:406-440): max_k |a_k - b_k| / |b_k|."""
    a = np.asarray(a, np.complex128)
    b = np.asarray(b, np.complex128)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-30)))


def vnorm_rel(a, b):
    a = np.asarray(a, np.complex128)
    b = np.asarray(b, np.complex128)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
