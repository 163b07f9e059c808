"""The tracking oracle (oracle/trk_oracle.c) against the reference's own unit-test
expectations, plus behavioural checks of the restated channel on synthetic IQ.

Pins: src/tests/unit-tests/signal-processing-blocks/tracking/
tracking_loop_filter_test.cc:22-206 (all six filter configurations) and
discriminator_test.cc:35-70 (BPSK early-minus-late).  The channel state machine
has no numeric golden vector in the reference; its behaviour is checked here
(pull-in, bit synchronisation, CN0 and Doppler of a known synthetic signal).
"""
import numpy as np
import pytest

from gsdr import synth
from oracle import trk

STEP = np.array([0.0, 0.0, 1.0, 0.0, 0.0, 0.0], np.float32)


@pytest.mark.parametrize("order,last,expected", [
    (1, False, [0.0, 0.0, 20.0, 0.0, 0.0, 0.0]),                       # :39-50 (g1 = 4 * 5)
    (1, True, [0.0, 0.0, 0.01, 0.02, 0.02, 0.02]),                     # :72
    (2, False, [0.0, 0.0, 13.37778, 0.0889, 0.0889, 0.0889]),          # :103
    (2, True, [0.0, 0.0, 0.006689, 0.013422, 0.013511, 0.013600]),     # :134
    (3, False, [0.0, 0.0, 15.31877, 0.04494, 0.04520, 0.04546]),       # :165
    (3, True, [0.0, 0.0, 0.007659, 0.015341, 0.015386, 0.015432]),     # :196
])
def test_loop_filter_golden(order, last, expected):
    got = trk.loop_filter_run(order, last, 5.0, 0.001, STEP)
    np.testing.assert_allclose(got, expected, atol=1e-4)


def test_dll_e_minus_l_bpsk_golden():
    """discriminator_test.cc:35-70: BPSK correlation 1-|tau|; output == err inside +-2*spacing."""
    for A in (1 + 0j, -1 + 0j, 1j, 1 + 1j):
        for spacing in (0.5, 0.25, 0.1, 0.01):
            for err in (0.0, 0.01, 0.1, 0.25, -0.25, -0.1, -0.01):
                bpsk = lambda x: 0.0 if abs(x) > 1.0 else 1.0 - abs(x)
                E = complex(np.complex64(A * np.float32(bpsk(err - spacing))))
                L = complex(np.complex64(A * np.float32(bpsk(err + spacing))))
                d = trk.dll_nc_e_minus_l_normalized(E, L, spacing, 1.0, 1.0)
                if abs(err) < 2.0 * spacing:
                    assert abs(d - err) <= 1e-4, (A, spacing, err, d)
                else:
                    assert err * d >= 0.0


def _conf(fs):
    c = trk.conf_default()
    c["fs_in"] = fs
    c["pll_bw_hz"] = 40.0   # conf/gnss-sdr_GPS_L1_gr_complex.conf:66-67
    c["dll_bw_hz"] = 4.0
    c["pull_in_time_s"] = 0  # leave pull-in after the first whole second
    return c


def test_channel_tracks_synthetic_gps_signal():
    fs = 2.0e6
    sat = synth.Satellite(7, 1234.5, 300.3, 45.0, 0.7, preamble_every_bits=50, code_doppler=True)
    iq = synth.gps_l1_iq(fs, int(3.2 * fs), [sat], seed_offset=5)
    ch = trk.Channel(_conf(fs))
    tau = sat.code_delay_chips / (1.023e6 * (1 + sat.doppler_hz / 1.57542e9)) * fs
    first = ch.start(synth.gps_ca_chips(7), float(round(tau)), 1250.0, 0, 2000)
    recs, _ = ch.run(iq, 0, first, 4000)
    assert len(recs) > 3000
    # states: pull-in (2) then bit synchronisation to narrow tracking (4)
    assert recs["state"][0] == 2 and recs["state"][-1] == 4
    sync = np.nonzero(recs["flags"] & trk.F_BIT_SYNC)[0]
    assert len(sync) == 1
    # consumption = one code period (+-1 sample) per call, contiguous input
    assert np.all(np.abs(recs["consumed"] - 2000) <= 1)
    assert np.all(np.diff(recs["sample_counter"].astype(np.int64)) == recs["consumed"][:-1])
    late = recs[-500:]
    assert abs(np.mean(late["carrier_doppler_hz"]) - sat.doppler_hz) < 2.0
    assert abs(np.mean(late["cn0_db_hz"]) - 45.0) < 1.5
    assert np.mean(late["carrier_lock_test"]) > 0.85
    # valid outputs: one per navigation bit (20 ms), prompt sign = the bit sign
    out = recs[(recs["flags"] & trk.F_VALID_OUTPUT) != 0]
    assert len(out) > 50
    assert np.all(np.abs(out["prompt_i"]) > 5 * np.abs(out["prompt_q"]))
    assert not np.any(recs["flags"] & trk.F_LOSS_OF_LOCK)


def test_channel_loses_lock_on_noise():
    """Noise only: the carrier lock detector fails (the m2m4 CN0 of pure noise sits
    near 26.7 dB-Hz, above cn0_min, so the code test passes) and, with a short
    max_carrier_lock_fail, the channel drops to state 0 with a loss-of-lock record
    (cn0_and_tracking_lock_status, :989-1025)."""
    fs = 2.0e6
    iq = synth.gps_l1_iq(fs, int(1.6 * fs), [], seed_offset=9)
    c = _conf(fs)
    c["max_carrier_lock_fail"] = 50
    ch = trk.Channel(c)
    first = ch.start(synth.gps_ca_chips(3), 100.0, 500.0, 0, 2000)
    recs, _ = ch.run(iq, 0, first, 4000)
    assert recs["flags"][-1] & trk.F_LOSS_OF_LOCK
    assert ch.state == 0


@pytest.mark.parametrize("at,cn0_fill", [(10, False), (300, True), (1300, True)])
def test_telemetry_fault_forces_loss_of_lock(at, cn0_fill):
    """msg_handler_telemetry_to_trk (dll_pll_veml_tracking.cc:614-637): the counter
    forced to 200000 fails the next lock check that evaluates the counters -- not
    before the CN0 buffer is full (:972-977, call 10 here waits for call 20) -- and
    the counters reset with the loss (:1022-1023).  The pull-in transitory ends at
    1 s (pull_in_time_s 0, integer seconds, :1797) and resets the counter too, so a
    fault in the transitory still fires at the next check inside it."""
    fs = 2.0e6
    sat = synth.Satellite(7, 1234.5, 300.3, 45.0, 0.7, preamble_every_bits=50, code_doppler=True)
    iq = synth.gps_l1_iq(fs, int(1.5 * fs), [sat], seed_offset=5)
    ch = trk.Channel(_conf(fs))
    tau = sat.code_delay_chips / (1.023e6 * (1 + sat.doppler_hz / 1.57542e9)) * fs
    first = ch.start(synth.gps_ca_chips(7), float(round(tau)), 1250.0, 0, 2000)
    a, n = ch.run(iq, 0, first, at)
    assert len(a) == at and not np.any(a["flags"] & trk.F_LOSS_OF_LOCK)
    ch.force_loss_of_lock()
    b, _ = ch.run(iq, 0, n, 4000)
    k = np.nonzero(b["flags"] & trk.F_LOSS_OF_LOCK)[0]
    assert len(k) == 1 and k[0] == len(b) - 1 and ch.state == 0
    # cn0_samples = 20: the first check that evaluates the counters is call 20
    assert at + k[0] == (at if cn0_fill else 20)


def _conf_sig(fs, sig, pilot=1):
    c = trk.conf_default()
    c["fs_in"] = fs
    c["signal"] = sig
    c["track_pilot"] = pilot
    c["pull_in_time_s"] = 0
    c["pll_bw_hz"] = 15.0
    c["dll_bw_hz"] = 1.0
    return c


@pytest.mark.parametrize("pilot", [1, 0])
def test_galileo_e1_channel(pilot):
    """Galileo E1 (dll_pll_veml_tracking.cc:258-290): VEML 5 taps on the sinBOC(1,1)
    replica at 2 samples/chip, 4 ms calls; pilot tracking locks the E1C secondary
    code after pull-in and reads the E1B data prompt from the extra correlator."""
    fs = 4.0e6
    sat = synth.GalileoSatellite(11, 1234.5, 1000.3, 50.0, 0.7)
    iq = synth.gal_e1_iq(fs, int(1.6 * fs), [sat], seed_offset=5)
    ch = trk.Channel(_conf_sig(fs, 1, pilot))
    assert ch.vector_length == 16000
    tau = sat.code_delay_chips / (1.023e6 * (1 + sat.doppler_hz / 1.57542e9)) * fs
    first = ch.start(synth.gal_e1_sinboc11(11, pilot=bool(pilot)), float(round(tau) % 16000), 1250.0, 0, 0, prn=11,
                     data_code=synth.gal_e1_sinboc11(11) if pilot else None)
    recs, _ = ch.run(iq, 0, first, 1000)
    assert len(recs) > 350 and recs["state"][-1] == 4
    sync = np.nonzero(recs["flags"] & trk.F_BIT_SYNC)[0]
    assert len(sync) == 1 and 249 <= sync[0] <= 249 + 26 * pilot
    assert np.all(np.abs(recs["consumed"] - 16000) <= 1)
    late = recs[-60:]
    assert abs(np.mean(late["carrier_doppler_hz"]) - sat.doppler_hz) < 3.0
    taps = late["taps"][:, :10].view(np.complex64)
    assert np.all(np.abs(taps[:, 2]) > np.abs(taps[:, 1])) and np.all(np.abs(taps[:, 2]) > np.abs(taps[:, 3]))
    out = recs[(recs["flags"] & trk.F_VALID_OUTPUT) != 0]
    assert len(out) == len(recs) - sync[0] - 1  # one 4 ms symbol per call after the lock
    tail = out[-60:]
    assert np.median(np.abs(tail["prompt_i"]) / (np.abs(tail["prompt_q"]) + 1e-9)) > 3.0
    if pilot:
        np.testing.assert_array_equal(tail["prompt_i"], tail["data_prompt"][:, 0].astype(np.float64))
    assert not np.any(recs["flags"] & trk.F_LOSS_OF_LOCK)


@pytest.mark.parametrize("prn,per", [(14, 20), (3, 2)])
def test_beidou_b1i_channel(prn, per):
    """BeiDou B1I (:391-411, :762-795): D1 satellites lock the NH code and emit one
    symbol per 20 ms with the NH wiped; D2 GEO satellites (PRN 1-5, 59-63) search
    the D2 preamble and emit one symbol per 2 ms."""
    fs = 4.0e6
    s = synth.Satellite(prn, -2262.3, 500.2, 45.0, 0.3)
    iq = synth.bds_b1i_iq(fs, int(1.6 * fs), [s], seed_offset=7)
    ch = trk.Channel(_conf_sig(fs, 2))
    assert ch.vector_length == 4000
    tau = s.code_delay_chips / (2.046e6 * (1 + s.doppler_hz / 1.561098e9)) * fs
    first = ch.start(synth.bds_b1i_chips(prn), float(round(tau) % 4000), -2250.0, 0, 0, prn=prn)
    recs, _ = ch.run(iq, 0, first, 1590)
    sync = np.nonzero(recs["flags"] & trk.F_BIT_SYNC)[0]
    assert len(sync) == 1 and recs["state"][-1] == 4
    assert abs(np.mean(recs[-100:]["carrier_doppler_hz"]) - s.doppler_hz) < 2.0
    out = np.nonzero(recs["flags"] & trk.F_VALID_OUTPUT)[0]
    assert len(out) > 5 and np.all(np.diff(out) == per)
    assert not np.any(recs["flags"] & trk.F_LOSS_OF_LOCK)


def test_extended_integration_cycle():
    """State 3 (dll_pll_veml_tracking.cc:1945-2026): after the secondary-code lock
    the channel alternates extend-1 accumulate-only calls (3) with one loop-update
    call (4) on the narrow loops and taps; Galileo E1 with 4 symbols (config C4)."""
    fs = 4.0e6
    c = _conf_sig(fs, 1, 1)
    c["extend_correlation_symbols"] = 4
    c["pll_bw_narrow_hz"] = 5.0
    c["dll_bw_narrow_hz"] = 0.25
    c["early_late_space_narrow_chips"] = 0.06
    c["very_early_late_space_narrow_chips"] = 0.25
    sat = synth.GalileoSatellite(11, 1234.5, 1000.3, 50.0, 0.7)
    iq = synth.gal_e1_iq(fs, int(1.6 * fs), [sat], seed_offset=5)
    ch = trk.Channel(c)
    tau = sat.code_delay_chips / (1.023e6 * (1 + sat.doppler_hz / 1.57542e9)) * fs
    first = ch.start(synth.gal_e1_sinboc11(11, pilot=True), float(round(tau) % 16000), 1250.0, 0, 0, prn=11,
                     data_code=synth.gal_e1_sinboc11(11))
    recs, _ = ch.run(iq, 0, first, 1000)
    sync = int(np.nonzero(recs["flags"] & trk.F_BIT_SYNC)[0][0])
    after = recs["state"][sync + 1:sync + 1 + 16]
    np.testing.assert_array_equal(after, [3, 3, 3, 4] * 4)
    assert np.all((recs["flags"][sync + 1:] & trk.F_VALID_OUTPUT) != 0)  # one 4 ms symbol per call
    assert abs(np.mean(recs[-60:]["carrier_doppler_hz"]) - sat.doppler_hz) < 2.0
    assert not np.any(recs["flags"] & trk.F_LOSS_OF_LOCK)


def test_log_data_points_and_dump(tmp_path):
    """log_data (dll_pll_veml_tracking.cc:1403-1500) is called in state 2 after every
    locked loop update and in states 3/4 when a data symbol completes; the engine
    flags those calls (TRK_F_LOGGED) and the dump file holds one 108-byte record for
    each.  Galileo E1 pilot with 4-symbol extended integration covers all three states."""
    import gsdr
    fs = 4.0e6
    c = _conf_sig(fs, 1, 1)
    c["extend_correlation_symbols"] = 4
    c["pll_bw_narrow_hz"] = 5.0
    c["dll_bw_narrow_hz"] = 0.25
    c["early_late_space_narrow_chips"] = 0.06
    c["very_early_late_space_narrow_chips"] = 0.25
    sat = synth.GalileoSatellite(11, 1234.5, 1000.3, 50.0, 0.7)
    iq = synth.gal_e1_iq(fs, int(1.2 * fs), [sat], seed_offset=5)
    ch = trk.Channel(c)
    tau = sat.code_delay_chips / (1.023e6 * (1 + sat.doppler_hz / 1.57542e9)) * fs
    first = ch.start(synth.gal_e1_sinboc11(11, pilot=True), float(round(tau) % 16000), 1250.0, 0, 0, prn=11,
                     data_code=synth.gal_e1_sinboc11(11))
    recs, _ = ch.run(iq, 0, first, 1000)
    logged = (recs["flags"] & trk.F_LOGGED) != 0
    lost = (recs["flags"] & trk.F_LOSS_OF_LOCK) != 0
    valid = (recs["flags"] & trk.F_VALID_OUTPUT) != 0
    want = ((recs["state"] == 2) & ~lost) | (np.isin(recs["state"], (3, 4)) & valid)
    np.testing.assert_array_equal(logged, want)
    assert np.count_nonzero(logged & (recs["state"] == 3)) > 10
    # state 2: the accumulators are the call's taps (VE, E, P, L, VL)
    s2 = recs[(recs["state"] == 2) & logged]
    taps = s2["taps"].reshape(-1, 5, 2)
    np.testing.assert_allclose(s2["log_accu"], np.hypot(taps[..., 0], taps[..., 1]), rtol=1e-6)
    # state 3 runs no loop update: its errors are the previous update's
    i3 = np.nonzero(recs["state"] == 3)[0]
    i3 = i3[i3 > 0]
    for f in ("carr_phase_error_hz", "code_error_chips", "code_error_filt_chips"):
        np.testing.assert_array_equal(recs[f][i3], recs[f][i3 - 1])
    assert np.all(recs["code_error_filt_chips"][recs["state"] == 4] != 0.0)
    # the dump records and their file round trip
    d = gsdr.trk_dump_records(recs, fs, 11, 123.25, 1250.0, veml=True, track_pilot=True)
    assert len(d) == np.count_nonzero(logged)
    path = tmp_path / "trk_dump11.dat"
    d.tofile(path)
    assert path.stat().st_size == 108 * len(d)
    back = gsdr.read_trk_dump(path)
    np.testing.assert_array_equal(back, d)
    r = recs[logged]
    np.testing.assert_array_equal(back["PRN_start_sample_count"], r["sample_counter"] + r["consumed"].astype(np.uint64))
    np.testing.assert_array_equal(back["Prompt_I"], r["data_prompt"][:, 0])
    np.testing.assert_array_equal(back["abs_P"], r["log_accu"][:, 2])
    np.testing.assert_array_equal(back["carr_error_hz"], r["carr_phase_error_hz"])
    assert np.all(back["PRN"] == 11) and np.all(back["acq_code_phase_samples"] == np.float32(123.25))
