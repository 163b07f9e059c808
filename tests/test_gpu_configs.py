"""Oracle parity of the device-resident tracking loop at every BASELINE.json
configuration's real rate and shape (the checks of test_gpu_trk.py -- open-loop
taps <= 1e-4 per call against the oracle correlator, replay of the GPU's taps
through the oracle loop with identical schedule / flags and bit-identical Prompt
I/Q, free-running agreement):

  C1/C2  GPS L1 C/A at 4 Msps (conf/gnss-sdr_GPS_L1_gr_complex.conf: PLL 40 Hz,
         DLL 4 Hz), one channel through bit synchronisation, gr_complex
  C3     GPS L1 C/A at 16 Msps, 12 channels in one pool launch
  C4     Galileo E1 at 8 Msps, ibyte input, E1-B/E1-C ICD memory codes, VEML with
         the data prompt, 4-symbol extended integration and the narrow taps of
         conf/gnss-sdr_galileo_E1_extended_correlator_byte.conf:98-110
  C5     one GPU's share of the 25 Msps hybrid pool: 12 GPS L1 C/A (N = 25000),
         12 Galileo E1 (N = 100000), 8 BeiDou B1I (N = 25000) on three handles over
         one IQ stream carrying all 32 satellites
"""
import json
import os

import numpy as np
import pytest

import gsdr
from gsdr import synth
from oracle import trk

from test_gpu_trk import (_conf, _conf_sig, _free_check, _open_loop_sig, _open_loop_taps, _replay_check)

pytestmark = pytest.mark.gpu


def _gps_acq(sat, fs):
    tau = sat.code_delay_chips / (1.023e6 * (1 + sat.doppler_hz / 1.57542e9)) * fs
    return float(round(tau) % round(fs / 1000)), float(250 * round(sat.doppler_hz / 250))


def _gal_acq(sat, fs):
    tau = sat.code_delay_chips / (1.023e6 * (1 + sat.doppler_hz / 1.57542e9)) * fs
    return float(round(tau) % round(fs / 250)), float(250 * round(sat.doppler_hz / 250))


def _bds_acq(sat, fs):
    tau = sat.code_delay_chips / (2.046e6 * (1 + sat.doppler_hz / 1.561098e9)) * fs
    return float(round(tau) % round(fs / 1000)), float(250 * round(sat.doppler_hz / 250))


def _pool_check(conf, sats, iq_host, iq_ref, fs, codes, data_codes, acq, max_epochs, tap_chips, spc, chip_rate, vl, iP,
                narrow=None, open_loop=None, tag="", free=True):
    """One pool launch of all channels, then per channel: open-loop taps, replay and
    free-running checks against an oracle channel with the same configuration."""
    spread = {}
    t = gsdr.Tracking(conf)
    starts = []
    for c, s in enumerate(sats):
        d, f = acq(s, fs)
        fg = t.start(c, s.prn, codes[c], d, f, 0, 0, data_code=None if data_codes is None else data_codes[c])
        starts.append((d, f, fg))
    rec, n = t.run(iq_host, 0, max_epochs)
    oc = conf[0:1].copy()
    oc["max_channels"] = 1
    oc = oc.view(trk.TRK_CONF_DTYPE)
    for c, s in enumerate(sats):
        d, f, fg = starts[c]
        g = rec[c][:n[c]]
        assert len(g) >= max_epochs // 2, (tag, c, len(g))
        dc = None if data_codes is None else data_codes[c]
        if open_loop is None or c in open_loop:
            worst = _open_loop_sig(g, iq_ref, codes[c], dc, fs, f, tap_chips, spc, chip_rate, vl, iP, narrow,
                                   spread=spread)
            assert worst <= 1e-4, (tag, c, worst)
        rep = trk.Channel(oc)
        assert rep.start(codes[c], d, f, 0, 0, prn=s.prn, data_code=dc) == fg
        _replay_check(g, rep, "%s ch%d" % (tag, c))
        if free:
            fr = trk.Channel(oc)
            fo = fr.start(codes[c], d, f, 0, 0, prn=s.prn, data_code=dc)
            orc, _ = fr.run(iq_ref, 0, fo, max_epochs)
            _free_check(g, orc, "%s ch%d" % (tag, c))
    _log_spread(tag, len(sats), spread)
    return rec, n


def _log_spread(tag, nch, spread):
    """Print (and with GSDR_PARITY_LOG append as JSON) the worst per-call distances
    of the GPU taps and of the generic VOLK correlator to the fp64 evaluation."""
    line = dict(tag=tag, channels=nch, **{k: (float(v) if isinstance(v, float) else v) for k, v in spread.items()})
    print("parity spread", json.dumps(line))
    path = os.environ.get("GSDR_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(line) + "\n")


def test_c1_c2_gps_4msps_through_bit_sync():
    fs = 4.0e6
    sat = synth.Satellite(7, 1234.5, 300.3, 45.0, 0.7, preamble_every_bits=25, code_doppler=True)
    iq = synth.gps_l1_iq(fs, int(1.7 * fs), [sat], seed_offset=31)
    d, f = _gps_acq(sat, fs)
    code = synth.gps_ca_chips(7)
    t = gsdr.Tracking(_conf(fs))
    fg = t.start(0, 7, code, d, f, 0, 0)
    rec, n = t.run(iq, 0, 1800)
    g = rec[0][:n[0]]
    assert _open_loop_taps(g, iq, code, fs, f) <= 1e-4
    oc = _conf(fs)[0:1].view(trk.TRK_CONF_DTYPE)
    rep = trk.Channel(oc)
    assert rep.start(code, d, f, 0, 0) == fg
    _replay_check(g, rep, "c2")
    fr = trk.Channel(oc)
    fo = fr.start(code, d, f, 0, 0)
    orc, _ = fr.run(iq, 0, fo, 1800)
    _free_check(g, orc, "c2")
    assert g["state"][-1] == 4 and np.any(g["flags"] & gsdr.TRK_F_BIT_SYNC)
    assert np.count_nonzero(g["flags"] & gsdr.TRK_F_VALID_OUTPUT) > 5
    assert abs(float(np.mean(g["carrier_doppler_hz"][-50:])) - sat.doppler_hz) < 2.0


def test_c3_gps_16msps_12_channel_pool():
    fs = 16.0e6
    # SURVEY §8(d)'s 45 dB-Hz.  Every call's taps are held to 1e-4 of the fp64
    # evaluation of the reference's correlation model (_open_loop_sig); the generic
    # VOLK rotator's own distance to that value is reported beside it
    sats = synth.random_constellation(12, seed_offset=33, cn0_dbhz=45.0)
    for s in sats:
        s.code_doppler = True
    iq = synth.gps_l1_iq(fs, int(0.2 * fs), sats, seed_offset=33)
    conf = _conf(fs, len(sats))
    codes = [synth.gps_ca_chips(s.prn) for s in sats]
    _pool_check(conf, sats, iq, iq, fs, codes, None, _gps_acq, 200, [-0.25, 0.0, 0.25], 1, 1.023e6, 16000, 1,
                tag="c3")


@pytest.mark.parametrize("fs", [16.384e6, 16.896e6, 16.897e6, 16.8965e6, 20.0e6, 24.6e6])
def test_streamed_chunk_tails(fs):
    """Streamed calls (vector_length > 4096) against the 8192-sample stream chunks of
    a GPS gr_complex pool: no tail (16384), a tail of exactly 512 samples riding with
    the last chunk (16896), one sample more -- a chunk of its own (16897) --, the same
    at a half-sample code period (16896.5: calls consume 16896 and 16897 samples in
    turn), a tail of several blocks (20000) and a short one behind three chunks (24600).  The
    chunk / tail split (csrc/trk.hip correlate_call_stream) must not change a sum."""
    sats = synth.random_constellation(2, seed_offset=37, cn0_dbhz=45.0)
    for s in sats:
        s.code_doppler = True
    iq = synth.gps_l1_iq(fs, int(0.06 * fs), sats, seed_offset=37)
    # the engine's vector_length: lround(fs / 1000), halves away from zero (16896.5 ->
    # 16897; consumption then alternates between 16896 and 16897 samples per call)
    vl = int(np.floor(fs / 1000 + 0.5))
    conf = _conf(fs, len(sats))
    codes = [synth.gps_ca_chips(s.prn) for s in sats]
    _pool_check(conf, sats, iq, iq, fs, codes, None, _gps_acq, 50, [-0.25, 0.0, 0.25], 1, 1.023e6, vl, 1,
                tag="tail%d" % vl)


def test_c4_galileo_8msps_ibyte_extended_veml():
    fs = 8.0e6
    # Dopplers within the narrow (15 Hz) PLL's pull-in of the 250 Hz acquisition grid
    # SURVEY §8(d)'s 45 dB-Hz (the pilot carries half of it)
    sats = [synth.GalileoSatellite(p, dop, dl, 45.0, ph) for p, dop, dl, ph in
            ((11, 1234.5, 1000.3, 0.7), (19, -2740.0, 3001.7, 2.1), (26, 505.0, 77.2, 4.0), (30, -995.0, 2500.9, 1.3))]
    x = synth.gal_e1_iq(fs, int(1.3 * fs), sats, seed_offset=35)
    host = synth.to_ibyte(x, 16.0)
    ref = synth.ibyte_to_complex(host)
    # conf/gnss-sdr_galileo_E1_extended_correlator_byte.conf:98-110
    c = _conf_sig(fs, gsdr.SIGNAL_GAL_1B, len(sats), 1)
    c["item_type"] = gsdr.ITEM_IBYTE
    c["pll_bw_hz"], c["dll_bw_hz"] = 15.0, 1.0
    c["pll_bw_narrow_hz"], c["dll_bw_narrow_hz"] = 5.0, 0.25
    c["early_late_space_chips"], c["very_early_late_space_chips"] = 0.15, 0.6
    c["early_late_space_narrow_chips"], c["very_early_late_space_narrow_chips"] = 0.06, 0.25
    c["extend_correlation_symbols"] = 4
    codes = [synth.gal_e1_sinboc11(s.prn, pilot=True) for s in sats]
    dcodes = [synth.gal_e1_sinboc11(s.prn) for s in sats]
    rec, n = _pool_check(c, sats, host, ref, fs, codes, dcodes, _gal_acq, 320, [-0.6, -0.15, 0.0, 0.15, 0.6], 2,
                         1.023e6, 32000, 2, narrow=[-0.25, -0.06, 0.0, 0.06, 0.25], tag="c4")
    for ch in range(len(sats)):
        st = set(np.unique(rec[ch][:n[ch]]["state"]).tolist())
        assert {2, 3, 4} <= st, (ch, st)


def test_c5_hybrid_25msps_pool_share():
    fs = 25.0e6
    ns = int(0.22 * fs)
    rng = np.random.default_rng(37)
    # SURVEY §8(d)'s 45 dB-Hz for every signal of the hybrid share
    gps = synth.random_constellation(12, seed_offset=37, cn0_dbhz=45.0)
    for s in gps:
        s.code_doppler = True
    gal_prns = rng.choice(np.arange(1, 37), 12, replace=False)
    gal = [synth.GalileoSatellite(int(p), float(rng.uniform(-4000, 4000)), float(rng.uniform(0, 4092)), 45.0,
                                  float(rng.uniform(0, 6.28))) for p in gal_prns]
    bds_prns = [3, 6, 8, 11, 14, 21, 33, 59]
    bds = [synth.Satellite(p, float(rng.uniform(-4000, 4000)), float(rng.uniform(0, 2046)), 45.0,
                           float(rng.uniform(0, 6.28))) for p in bds_prns]
    iq = (synth.gps_l1_iq(fs, ns, gps, seed_offset=37, noise=False, dtype=np.complex128) +
          synth.gal_e1_iq(fs, ns, gal, seed_offset=37, noise=False, dtype=np.complex128) +
          synth.bds_b1i_iq(fs, ns, bds, seed_offset=37, noise=True, dtype=np.complex128)).astype(np.complex64)
    # GPS L1 C/A, N = 25000
    _pool_check(_conf(fs, 12), gps, iq, iq, fs, [synth.gps_ca_chips(s.prn) for s in gps], None, _gps_acq, 215,
                [-0.25, 0.0, 0.25], 1, 1.023e6, 25000, 1, tag="c5gps")
    # Galileo E1 pilot tracking, N = 100000
    _pool_check(_conf_sig(fs, gsdr.SIGNAL_GAL_1B, 12, 1), gal, iq, iq, fs,
                [synth.gal_e1_sinboc11(s.prn, pilot=True) for s in gal], [synth.gal_e1_sinboc11(s.prn) for s in gal],
                _gal_acq, 53, [-0.5, -0.25, 0.0, 0.25, 0.5], 2, 1.023e6, 100000, 2, tag="c5gal")
    # BeiDou B1I (D1 and D2 GEO), N = 25000
    _pool_check(_conf_sig(fs, gsdr.SIGNAL_BDS_B1, 8), bds, iq, iq, fs, [synth.bds_b1i_chips(s.prn) for s in bds], None,
                _bds_acq, 215, [-0.25, 0.0, 0.25], 1, 2.046e6, 25000, 1, tag="c5bds")
