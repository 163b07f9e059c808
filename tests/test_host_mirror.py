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


def test_tracking_dump_matfile_reads_back(tmp_path):
    """save_matfile (dll_pll_veml_tracking.cc:1511-1729): the .dat records of a channel
    converted into <stem><channel>.mat with the reference's 25 variables, their
    classes and 1 x epochs shape, values equal to the .dat fields (CPU, no HIP)."""
    sio = pytest.importorskip("scipy.io")
    exe = os.path.join(BUILD, "trk_mat_probe")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", HOST, exe])
    subprocess.check_call([exe, str(tmp_path)])
    raw = np.fromfile(str(tmp_path / "trk_dump5.dat"), np.uint8)
    assert raw.size == 37 * 108
    rec = np.dtype([("f1", "<f4", 7), ("stamp", "<u8"), ("f2", "<f4", 12), ("aux2", "<f8"), ("prn", "<u4"),
                    ("f3", "<f4", 3)])
    assert rec.itemsize == 108
    d = raw.view(rec)
    m = sio.loadmat(str(tmp_path / "trk_dump5.mat"))
    names1 = ["abs_VE", "abs_E", "abs_P", "abs_L", "abs_VL", "Prompt_I", "Prompt_Q"]
    names2 = ["acc_carrier_phase_rad", "carrier_doppler_hz", "carrier_doppler_rate_hz", "code_freq_chips",
              "code_freq_rate_chips", "carr_error_hz", "carr_error_filt_hz", "code_error_chips", "code_error_filt_chips",
              "CN0_SNV_dB_Hz", "carrier_lock_test", "aux1"]
    names3 = ["acq_code_phase_samples", "acq_carrier_doppler_hz", "EVM"]
    assert sorted(k for k in m if not k.startswith("__")) == sorted(names1 + names2 + names3 + [
        "PRN_start_sample_count", "aux2", "PRN"])
    for k, nm in enumerate(names1):
        assert m[nm].dtype == np.float32 and m[nm].shape == (1, 37)
        np.testing.assert_array_equal(m[nm][0], d["f1"][:, k])
    for k, nm in enumerate(names2):
        assert m[nm].dtype == np.float32
        np.testing.assert_array_equal(m[nm][0], d["f2"][:, k])
    for k, nm in enumerate(names3):
        np.testing.assert_array_equal(m[nm][0], d["f3"][:, k])
    assert m["PRN_start_sample_count"].dtype == np.uint64 and m["aux2"].dtype == np.float64
    np.testing.assert_array_equal(m["PRN_start_sample_count"][0], d["stamp"])
    np.testing.assert_array_equal(m["aux2"][0], d["aux2"])
    assert m["PRN"].dtype == np.uint32 and np.all(m["PRN"][0] == 17)
    # the probe's values: |E| of record i, VEML taps
    np.testing.assert_array_equal(m["abs_E"][0], 100.0 * np.arange(37) + 1.0)


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
    on the device ring -- every channel converges, emits Gnss_Synchro items after the
    pull-in, and the searched PRNs are answered."""
    import json
    exe = os.path.join(BUILD, "receiver_bench")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", HOST, exe])
    # 1.6 s: past the 1 s pull-in transitory (dll_pll_veml_tracking.cc:1797) and the
    # bit synchronisation, so every channel reaches state 4 and emits
    r = subprocess.run([exe, "c3", "1.6"], capture_output=True, text=True, timeout=240)
    print(r.stdout, r.stderr[-2000:])
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    g = d["signals"]["G1C"]
    assert g["channels"] == 12 and g["channels_within_25hz"] == 12, d
    assert g["channels_with_outputs"] == 12 and g["min_outputs_per_channel"] > 0, d
    assert g["acq_answers"] > 0, d  # the untracked PRNs keep being searched (pfa 0.01: rare false alarms)
    assert d["msps"] > 0


def _parse_synchro(path):
    acq, tags, outs = None, [], []
    for line in open(path):
        f = line.split()
        if f[0] == "acq":
            acq = dict(prn=int(f[1]), ch=int(f[2]), delay=float(f[3]), dop=float(f[4]), stamp=int(f[5]),
                       pi=float(f[6]), pq=float(f[7]), cn0=float(f[8]), cdop=float(f[9]), corr=int(f[10]))
        elif f[0] == "tag":
            tags.append((int(f[1]), int(f[2]), int(f[3]), float(f[4])))
        elif f[0] == "out":
            o = dict(prn=int(f[1]), ch=int(f[2]), sig=f[3], delay=float(f[4]), dop=float(f[5]), stamp=int(f[6]),
                     fs=int(f[7]), pi=float(f[8]), pq=float(f[9]), cn0=float(f[10]), cdop=float(f[11]),
                     phase=float(f[12]), code=float(f[13]), tsc=int(f[14]), corr=int(f[15]), evm=float(f[16]),
                     valid=int(f[17]), pll180=int(f[18]), vacq=int(f[19]), tag=None)
            if len(f) > 20:
                o["tag"] = (int(f[21]), int(f[22]), int(f[23]), float(f[24]), float(f[25]))
            outs.append(o)
    return acq, tags, outs


def _expected_tags(recs, emits, tags, fs):
    """The time-tag part of general_work (dll_pll_veml_tracking.cc:2088-2147),
    restated: every call keeps the last tag of [nitems_read, nitems_read +
    consumed); an output re-emits it at output item nitems_written + 1 with the tow
    advanced by the (signed) sample distance."""
    import math
    import gsdr
    out, waiting, last, written = [], False, None, 0
    for r in recs:
        sc, n = int(r["sample_counter"]), int(r["consumed"])
        for t in tags:
            if sc <= t[0] < sc + n:
                last, waiting = [t[0], t[1], t[2], t[3]], True
        if not (int(r["flags"]) & (gsdr.TRK_F_VALID_OUTPUT | gsdr.TRK_F_LOSS_OF_LOCK)):
            continue
        tag = None
        if waiting:
            frac, intpart = math.modf(1000.0 * float(sc - last[0]) / fs)
            last[3] = last[3] + frac
            tag = (written + 1, last[1], last[2] + int(intpart), last[3], sc / fs)
            waiting = False
        out.append(tag)
        written += 1
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["channel", "pooled"])
def test_gnss_synchro_emission_matches_oracle(tmp_path, kind):
    """Both tracking blocks' Gnss_Synchro items against the reference's general_work
    (dll_pll_veml_tracking.cc:1784-2152), field by field: valid outputs carry the
    call's Prompt/CN0/Doppler/phases and correlation_length_ms 1 (GPS L1 C/A, :178);
    the telemetry fault (msg_handler_telemetry_to_trk, :614-637) ends in ONE loss-of-lock
    item that is the acquisition record (:1878, :2040) with fs, the sample counter and
    the flags of :2121-2127; the output time tags follow :2088-2147.  The records
    replayed through the oracle channel with the fault before the same call reproduce
    the schedule, flags and prompts."""
    import gsdr
    from oracle import trk
    exe = os.path.join(BUILD, "host_selftest")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", HOST])
    d = os.environ.get("GSDR_SYNCHRO_DIR")
    if not d:
        cap = os.path.join(ROOT, "tests", "golden", "GPS_L1_CA_ID_1_Fs_4Msps_2ms.dat")
        env = dict(os.environ, GSDR_SELFTEST_DUMP_DIR=str(tmp_path), GSDR_SELFTEST_ONLY="synchro")
        r = subprocess.run([exe, cap], capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        d = str(tmp_path)
    fs = 4000000.0
    acq, tags, outs = _parse_synchro(os.path.join(d, "synchro_%s.txt" % kind))
    recs = np.fromfile(os.path.join(d, "synchro_%s.recs" % kind), gsdr.TRK_EPOCH_DTYPE)
    flags = recs["flags"].astype(np.int64)
    emit = np.nonzero(flags & (gsdr.TRK_F_VALID_OUTPUT | gsdr.TRK_F_LOSS_OF_LOCK))[0]
    assert len(outs) == len(emit) and len(outs) > 20
    lol = np.nonzero(flags & gsdr.TRK_F_LOSS_OF_LOCK)[0]
    assert len(lol) == 1 and lol[0] == len(recs) - 1  # the fault's call ends the run
    for k, o in zip(emit, outs):
        r = recs[k]
        assert o["tsc"] == int(r["sample_counter"]) and o["fs"] == 4000000
        assert o["prn"] == acq["prn"] and o["ch"] == acq["ch"] and o["sig"] == "1C" and o["vacq"] == 1
        assert o["delay"] == acq["delay"] and o["dop"] == acq["dop"] and o["stamp"] == acq["stamp"]
        assert o["pll180"] == int(bool(int(r["flags"]) & gsdr.TRK_F_PLL_180))
        if int(r["flags"]) & gsdr.TRK_F_LOSS_OF_LOCK:
            # the acquisition record, none of the call's tracking values
            assert o["valid"] == 0 and o["pi"] == acq["pi"] and o["pq"] == acq["pq"] and o["cn0"] == acq["cn0"]
            assert o["cdop"] == acq["cdop"] and o["corr"] == acq["corr"] and o["phase"] == 0.0 and o["evm"] == 0.0
        else:
            assert o["valid"] == 1 and o["corr"] == 1
            assert o["pi"] == float(r["prompt_i"]) and o["pq"] == float(r["prompt_q"])
            assert o["cn0"] == float(r["cn0_db_hz"]) and o["cdop"] == float(r["carrier_doppler_hz"])
            assert o["phase"] == float(r["acc_carrier_phase_rad"]) and o["code"] == float(r["rem_code_phase_samples"])
            assert o["evm"] == float(r["evm"])
    exp = _expected_tags(recs, emit, tags, fs)
    got = [o["tag"] for o in outs]
    assert sum(t is not None for t in exp) >= 5
    for e, g in zip(exp, got):
        assert (e is None) == (g is None)
        if e is not None:
            assert g[0] == e[0] and g[1] == e[1] and g[2] == e[2]
            assert abs(g[3] - e[3]) <= 1e-9 and abs(g[4] - e[4]) <= 1e-9
    # the oracle channel with the same start and the fault before the same call
    c = trk.conf_default()
    c["fs_in"], c["pll_bw_hz"], c["dll_bw_hz"], c["pull_in_time_s"], c["max_channels"] = fs, 40.0, 4.0, 0, 1
    # both blocks ran their pull-in (state 1) on the first work() call, at nitems_read 0
    first = ch_first = None
    ch = trk.Channel(c)
    ch_first = ch.start(replica.gps_l1_ca_code_float(1), acq["delay"], acq["dop"], acq["stamp"], 0, prn=1)
    first = int(recs["sample_counter"][0])
    assert ch_first == first
    o = ch.replay(recs, force_before=[int(lol[0])])
    for f in ("sample_counter", "consumed", "state", "flags"):
        np.testing.assert_array_equal(recs[f], o[f], err_msg=f)
    np.testing.assert_array_equal(recs["prompt_i"], o["prompt_i"])
    np.testing.assert_array_equal(recs["prompt_q"], o["prompt_q"])
