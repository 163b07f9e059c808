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


def test_mat5_writer_reads_back(tmp_path):
    """The acquisition dump's Level-5 MAT-file writer (host/mat5_writer.cc): names,
    classes, dimensions and column-major data as scipy.io.loadmat reads them."""
    sio = pytest.importorskip("scipy.io")
    exe = os.path.join(BUILD, "mat5_probe")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", HOST, exe])
    path = tmp_path / "probe.mat"
    subprocess.check_call([exe, str(path)])
    m = sio.loadmat(str(path))
    g = m["acq_grid"]
    assert g.dtype == np.float32 and g.shape == (5, 3)
    np.testing.assert_array_equal(g, np.arange(5)[:, None] + 0.25 * np.arange(3)[None, :])
    assert m["doppler_max"].dtype == np.int32 and int(m["doppler_max"][0, 0]) == -5000
    assert m["test_statistic"].dtype == np.float32 and float(m["test_statistic"][0, 0]) == 3.5
    assert m["PRN"].dtype == np.uint32 and int(m["PRN"][0, 0]) == 17
    assert m["sample_counter"].dtype == np.uint64 and int(m["sample_counter"][0, 0]) == 123456789012345


@pytest.mark.gpu
def test_host_selftest_on_gpu(tmp_path):
    exe = os.path.join(BUILD, "host_selftest")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", HOST])
    cap = os.path.join(ROOT, "tests", "golden", "GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat")
    gal = os.path.join(ROOT, "tests", "golden", "Galileo_E1_ID_1_Fs_4Msps_8ms.dat")
    env = dict(os.environ, GSDR_SELFTEST_DUMP_DIR=str(tmp_path))
    r = subprocess.run([exe, cap, gal], capture_output=True, text=True, timeout=120, env=env)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_selftest: PASS" in r.stdout
    _check_acq_dumps(tmp_path, cap)


def _check_acq_dumps(d, cap_path):
    """The acquisition dump files the self-test wrote (dump_results,
    pcps_acquisition.cc:408-508) against the oracle grid of the same block."""
    sio = pytest.importorskip("scipy.io")
    from oracle import pcps
    x = np.fromfile(cap_path, np.complex64)
    fs, N = 4000000, 4000
    code = replica.gps_l1_ca_code_complex_sampled(1, fs)
    cf = pcps.fft_code(code, N, N)
    # single step: +-5 kHz / 100 Hz on the first millisecond
    m = sio.loadmat(str(d / "acq_one_G_1C_ch_1_1_sat_1.mat"))
    M = pcps.magnitude_grid(x[:N], pcps.doppler_wipeoffs(fs, N, 5000, 100, 100), cf)  # D x N
    g = m["acq_grid"]
    assert g.shape == (N, 100) and g.dtype == np.float32
    assert np.max(np.abs(g.T - M)) <= 1e-4 * M.max()
    ti, di, gmax, ip, stat = pcps.max_to_input_power_statistic(M)
    assert abs(float(m["test_statistic"][0, 0]) - stat) <= 1e-4 * stat
    assert int(m["PRN"][0, 0]) == 1 and int(m["num_dwells"][0, 0]) == 1 and int(m["d_positive_acq"][0, 0]) == 1
    assert int(m["doppler_max"][0, 0]) == 5000 and int(m["doppler_step"][0, 0]) == 100
    assert int(m["sample_counter"][0, 0]) == N
    assert abs(float(m["acq_delay_samples"][0, 0]) - 524) * 1023 / fs < 0.5
    # two steps: the narrow 5 x 100 Hz grid around the coarse Doppler on the second millisecond
    m = sio.loadmat(str(d / "acq_two_G_1C_ch_1_1_sat_1.mat"))
    assert m["acq_grid"].shape == (N, 20) and m["acq_grid_narrow"].shape == (N, 5)
    step2, lo = float(m["doppler_step_narrow"][0, 0]), float(m["doppler_grid_narrow_min"][0, 0])
    assert step2 == 100.0
    center = lo + 2 * step2
    Mn = pcps.magnitude_grid(x[N:2 * N], pcps.doppler_wipeoffs_step2(fs, N, center, step2, 5), cf)
    assert np.max(np.abs(m["acq_grid_narrow"].T - Mn)) <= 1e-4 * Mn.max()


@pytest.mark.gpu
def test_receiver_bench_c3_tracks_every_channel():
    """The drop-in receiver path at config C3's scale (host/tests/receiver_bench.cc):
    12 factory-built pooled tracking blocks at 16 Msps beside the acquisition service
    on the device ring -- every channel converges and the searched PRNs are answered."""
    import json
    exe = os.path.join(BUILD, "receiver_bench")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", HOST, exe])
    r = subprocess.run([exe, "c3", "0.15"], capture_output=True, text=True, timeout=180)
    print(r.stdout, r.stderr[-2000:])
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    g = d["signals"]["G1C"]
    assert g["channels"] == 12 and g["channels_within_25hz"] == 12, d
    assert g["acq_answers"] > 0, d  # the untracked PRNs keep being searched (pfa 0.01: rare false alarms)
    assert d["msps"] > 0
