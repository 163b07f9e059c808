"""ORACLE — test infrastructure only.  ctypes front-end of oracle/trk_oracle.c,
the CPU restatement of dll_pll_veml_tracking (GPS L1 C/A, Galileo E1, BeiDou B1I)
and its loop library."""
import ctypes

import numpy as np

from . import volk

_d = ctypes.c_double
_f = ctypes.c_float
_i = ctypes.c_int
_p = ctypes.c_void_p
_u64 = ctypes.c_uint64

# include/gsdr.h: gsdr_trk_conf / gsdr_trk_epoch (C layout, natural alignment)
TRK_CONF_DTYPE = np.dtype([
    ("fs_in", "f8"), ("carrier_lock_th", "f8"), ("vector_length", "u4"), ("signal", "i4"), ("item_type", "i4"),
    ("max_channels", "u4"), ("fll_bw_hz", "f4"), ("pll_bw_hz", "f4"), ("dll_bw_hz", "f4"), ("pll_bw_narrow_hz", "f4"),
    ("dll_bw_narrow_hz", "f4"), ("early_late_space_chips", "f4"), ("very_early_late_space_chips", "f4"),
    ("early_late_space_narrow_chips", "f4"), ("very_early_late_space_narrow_chips", "f4"),
    ("cn0_smoother_alpha", "f4"), ("carrier_lock_test_smoother_alpha", "f4"), ("pull_in_time_s", "u4"),
    ("bit_synchronization_time_limit_s", "u4"), ("pll_filter_order", "i4"), ("dll_filter_order", "i4"),
    ("extend_correlation_symbols", "i4"), ("cn0_samples", "i4"), ("cn0_smoother_samples", "i4"),
    ("carrier_lock_test_smoother_samples", "i4"), ("cn0_min", "i4"), ("max_code_lock_fail", "i4"),
    ("max_carrier_lock_fail", "i4"), ("enable_fll_pull_in", "i4"), ("enable_fll_steady_state", "i4"),
    ("carrier_aiding", "i4"), ("high_dyn", "i4"), ("track_pilot", "i4"), ("smoother_length", "u4")], align=True)
assert TRK_CONF_DTYPE.itemsize == 144

TRK_EPOCH_DTYPE = np.dtype([
    ("sample_counter", "u8"), ("state", "i4"), ("consumed", "i4"), ("taps", "f4", (10,)),
    ("rem_carr_phase_rad", "f4"), ("flags", "i4"), ("carrier_doppler_hz", "f8"), ("code_freq_chips", "f8"),
    ("rem_code_phase_samples", "f8"), ("acc_carrier_phase_rad", "f8"), ("cn0_db_hz", "f8"),
    ("carrier_lock_test", "f8"), ("prompt_i", "f8"), ("prompt_q", "f8"), ("evm", "f8"), ("data_prompt", "f4", (2,)),
    ("carrier_rate", "f4"), ("code_rate", "f4"), ("log_accu", "f4", (5,)), ("carr_phase_error_hz", "f4"),
    ("carr_error_filt_hz", "f4"), ("code_error_chips", "f4"), ("code_error_filt_chips", "f4"), ("reserved", "i4")], align=True)
assert TRK_EPOCH_DTYPE.itemsize == 192

F_VALID_OUTPUT, F_LOSS_OF_LOCK, F_PLL_180, F_BIT_SYNC, F_LOGGED = 1, 2, 4, 8, 32

_init = False


def _lib():
    global _init
    L = volk.lib()
    if not _init:
        L.orc_trk_conf_default.argtypes = [_p]
        L.orc_trk_create.argtypes = [_p]
        L.orc_trk_create.restype = _p
        L.orc_trk_destroy.argtypes = [_p]
        L.orc_trk_set_assoc.argtypes = [_p, _i]
        L.orc_trk_start.argtypes = [_p, ctypes.c_uint32, _p, _i, _d, _d, _u64, _u64, _p]
        L.orc_trk_set_data_code.argtypes = [_p, _p, _i]
        L.orc_trk_set_data_code.restype = _i
        L.orc_trk_start.restype = _i
        L.orc_trk_call.argtypes = [_p, _p, _u64, _p]
        L.orc_trk_call.restype = _i
        L.orc_trk_call_taps.argtypes = [_p, _p, _u64, _p]
        L.orc_trk_call_taps.restype = _i
        L.orc_trk_force_loss_of_lock.argtypes = [_p]
        L.orc_trk_state.argtypes = [_p]
        L.orc_trk_state.restype = ctypes.c_int32
        L.orc_trk_vector_length.argtypes = [_p]
        L.orc_trk_vector_length.restype = ctypes.c_int32
        L.orc_loop_filter_run.argtypes = [_i, _i, _f, _f, _p, _p, _i]
        L.orc_dll_nc_e_minus_l_normalized.argtypes = [_f, _f, _f, _f, _f, _f, _f]
        L.orc_dll_nc_e_minus_l_normalized.restype = _d
        _init = True
    return L


def conf_default():
    c = np.zeros(1, TRK_CONF_DTYPE)
    _lib().orc_trk_conf_default(c.ctypes.data)
    return c


def loop_filter_run(order, last_int, bw, T, x):
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    _lib().orc_loop_filter_run(order, int(last_int), bw, T, x.ctypes.data, out.ctypes.data, len(x))
    return out


def dll_nc_e_minus_l_normalized(E, L, spc=0.5, slope=1.0, y_intercept=1.0):
    return _lib().orc_dll_nc_e_minus_l_normalized(E.real, E.imag, L.real, L.imag, spc, slope, y_intercept)


class Channel:
    """One dll_pll_veml_tracking channel (GPS L1 C/A, Galileo E1, BeiDou B1I)."""

    def __init__(self, conf):
        self._conf = np.ascontiguousarray(conf, TRK_CONF_DTYPE)
        self._h = _lib().orc_trk_create(self._conf.ctypes.data)
        if not self._h:
            raise ValueError("configuration not supported by the oracle")

    def __del__(self):
        if getattr(self, "_h", None):
            _lib().orc_trk_destroy(self._h)
            self._h = None

    @property
    def vector_length(self):
        return int(_lib().orc_trk_vector_length(self._h))

    @property
    def state(self):
        return int(_lib().orc_trk_state(self._h))

    def set_assoc(self, assoc):
        _lib().orc_trk_set_assoc(self._h, assoc)

    def start(self, code, acq_delay_samples, acq_doppler_hz, acq_samplestamp, nitems_read, prn=1, data_code=None):
        code = np.ascontiguousarray(code, np.float32)
        if data_code is not None:
            dc = np.ascontiguousarray(data_code, np.float32)
            if _lib().orc_trk_set_data_code(self._h, dc.ctypes.data, len(dc)) != 0:
                raise ValueError("bad data code replica")
        first = ctypes.c_uint64()
        rc = _lib().orc_trk_start(self._h, int(prn), code.ctypes.data, len(code), acq_delay_samples, acq_doppler_hz,
                                  acq_samplestamp, nitems_read, ctypes.byref(first))
        if rc != 0:
            raise ValueError("bad code replica")
        return int(first.value)

    def run(self, iq, iq_first_sample, first_sample, max_epochs):
        """Drive general_work over iq (complex64, absolute index iq_first_sample)
        from first_sample; returns the records."""
        iq = np.ascontiguousarray(iq, np.complex64)
        vl = self.vector_length
        recs = np.zeros(max_epochs, TRK_EPOCH_DTYPE)
        n = first_sample
        k = 0
        while k < max_epochs:
            off = n - iq_first_sample
            if off < 0 or off + vl > len(iq):
                break
            r = recs[k:k + 1]
            if not _lib().orc_trk_call(self._h, iq[off:].ctypes.data, n, r.ctypes.data):
                break
            n += int(r["consumed"][0])
            k += 1
        return recs[:k], n

    def force_loss_of_lock(self):
        """msg_handler_telemetry_to_trk with a telemetry fault (:614-637)."""
        _lib().orc_trk_force_loss_of_lock(self._h)

    def replay(self, records, force_before=()):
        """Feed the correlator outputs of another implementation's records through
        this channel's loop (orc_trk_call_taps), call by call at the same input
        positions; returns this channel's own records.  force_before: record
        indices before which a telemetry fault arrives (force_loss_of_lock)."""
        out = np.zeros(len(records), TRK_EPOCH_DTYPE)
        force = set(int(i) for i in force_before)
        for k, rec in enumerate(records):
            if k in force:
                self.force_loss_of_lock()
            taps = np.concatenate([rec["taps"], rec["data_prompt"]]).astype(np.float32)
            if not _lib().orc_trk_call_taps(self._h, taps.ctypes.data, int(rec["sample_counter"]), out[k:k + 1].ctypes.data):
                return out[:k]
        return out
