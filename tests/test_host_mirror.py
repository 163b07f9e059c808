"""Host-side C++ mirror (gnss-sdr-new_amd/host/): CPU checks of the replica
generator and Acq_Conf restatement against the oracle, and the GPU self-test of
the adapter / block / correlator drop-ins (written like the reference's tests)."""
import os
import subprocess

import numpy as np
import pytest

from oracle import replica

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "gnss-sdr-new_amd", "host")
BUILD = os.path.join(ROOT, "gnss-sdr-new_amd", "build")

PROBE = r'''
#include <cstdio>
#include "gnss_replicas.h"
#include "acq_conf.h"
int main() {
  for (int prn = 1; prn <= 32; ++prn) {
    auto c = gps_l1_ca_code_gen_int(prn, 0);
    for (int v : c) std::printf("%d ", v);
    std::printf("\n");
  }
  for (int fs : {2000000, 4000000, 6625000, 8000000}) {
    auto s = gps_l1_ca_code_gen_complex_sampled(7, fs, 0);
    for (auto& v : s) std::printf("%d ", (int)v.imag());
    std::printf("\n");
  }
  InMemoryConfiguration cfg;
  cfg.set_property("GNSS-SDR.internal_fs_sps", "4000000");
  cfg.set_property("Acquisition_1C.pfa", "0.01");
  cfg.set_property("Acquisition_1C.doppler_max", "10000");
  Acq_Conf a; a.SetFromConfiguration(&cfg, "Acquisition_1C", 1023000.0, 2000000.0);
  std::printf("%lld %u %.17g %.17g %d %d %d\n", (long long)a.fs_in, a.samples_per_chip, a.samples_per_ms,
              a.samples_per_code, a.doppler_max, (int)a.use_CFAR_algorithm_flag, (int)a.it_size);
  return 0;
}
'''


def test_cpp_replica_and_acq_conf_match_oracle(tmp_path):
    src = tmp_path / "probe.cc"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-ffp-contract=off", "-I", HOST, "-I",
                           os.path.join(ROOT, "include"), "-Wa,-I" + os.path.join(ROOT, "gnss-sdr-new_amd", "gsdr", "data"),
                           str(src), os.path.join(HOST, "gnss_replicas.cc"), os.path.join(HOST, "galileo_e1_codes.cc"),
                           os.path.join(HOST, "acq_conf.cc"), "-o", str(exe)])
    lines = subprocess.check_output([str(exe)], text=True).splitlines()
    for prn in range(1, 33):
        got = np.array(lines[prn - 1].split(), np.int32)
        np.testing.assert_array_equal(got, replica.gps_l1_ca_code_int(prn))
    for i, fs in enumerate((2000000, 4000000, 6625000, 8000000)):
        got = np.array(lines[32 + i].split(), np.int32)
        np.testing.assert_array_equal(got, replica.gps_l1_ca_code_complex_sampled(7, fs).imag.astype(np.int32))
    f = lines[36].split()
    spms = float(np.float32(4000000) * np.float32(0.001))  # 4000.00024: the reference's float arithmetic
    assert f[0] == "4000000" and f[1] == "4" and float(f[2]) == spms and float(f[3]) == spms
    assert f[4] == "10000" and f[5] == "1" and f[6] == "8"


@pytest.mark.gpu
def test_host_selftest_on_gpu():
    exe = os.path.join(BUILD, "host_selftest")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", HOST])
    cap = os.path.join(ROOT, "tests", "golden", "GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat")
    gal = os.path.join(ROOT, "tests", "golden", "Galileo_E1_ID_1_Fs_4Msps_8ms.dat")
    r = subprocess.run([exe, cap, gal], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_selftest: PASS" in r.stdout
