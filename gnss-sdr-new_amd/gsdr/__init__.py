"""Python front-end of libgsdr.so (the MI355X acquisition + tracking correlator
engine).  Thin ctypes layer over the C ABI declared in include/gsdr.h; used by the
tests, bench.py and __graft_entry__.  It has no compute of its own and no CPU
fallback: if the HIP library cannot be loaded, every entry point raises.
"""
import contextlib
import ctypes
import os

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GSDR_LIB", os.path.join(_PKG, "build", "libgsdr.so"))

GSDR_OK = 0
GSDR_E_ARG = -1
GSDR_E_DEVICE = -2
GSDR_E_ALLOC = -3
GSDR_E_STATE = -4
GSDR_E_UNSUPPORTED = -5

ITEM_GR_COMPLEX = 0
ITEM_CSHORT = 1
ITEM_IBYTE = 2  # interleaved int8 I,Q (Ibyte_To_Complex)
_ITEM_NP = {0: np.complex64, 1: np.int16, 2: np.int8}
ASSOC_GENERIC = 0
ASSOC_AVX = 1

# Every symbol include/gsdr.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "gsdr_last_error", "gsdr_abi_version", "gsdr_device_count",
    "gsdr_acq_create", "gsdr_acq_destroy", "gsdr_acq_get_dims", "gsdr_acq_set_local_codes",
    "gsdr_acq_set_doppler", "gsdr_acq_set_threshold", "gsdr_acq_get_threshold", "gsdr_acq_run",
    "gsdr_acq_run_device", "gsdr_acq_dump_grid", "gsdr_acq_dump_spectra", "gsdr_acq_set_profiling",
    "gsdr_acq_read_profile",
    "gsdr_corr_create", "gsdr_corr_destroy", "gsdr_corr_set_local_code_and_taps",
    "gsdr_corr_set_local_code_and_taps_complex", "gsdr_corr_set_high_dynamics_resampler",
    "gsdr_corr_set_resampler_assoc", "gsdr_corr_run", "gsdr_corr_run_batch", "gsdr_corr_run_batch_device",
    "gsdr_corr_dump_indices", "gsdr_corr_run_epochs", "gsdr_corr_set_profiling", "gsdr_corr_read_profile",
    "gsdr_trk_conf_default", "gsdr_trk_create", "gsdr_trk_destroy", "gsdr_trk_start", "gsdr_trk_stop",
    "gsdr_trk_run_device", "gsdr_trk_run", "gsdr_trk_get_channel", "gsdr_trk_save_state", "gsdr_trk_restore_state",
    "gsdr_trk_set_profiling", "gsdr_trk_read_profile", "gsdr_acq_set_cu_mask", "gsdr_trk_set_cu_mask",
    "gsdr_acq_run_dwell", "gsdr_acq_run_stream", "gsdr_trk_run_stream", "gsdr_trk_run_stream_host",
    "gsdr_stream_create", "gsdr_stream_destroy", "gsdr_stream_push", "gsdr_stream_span", "gsdr_stream_window",
    "gsdr_acq_set_step_two", "gsdr_acq_get_step_two_threshold", "gsdr_acq_run_step_two",
    "gsdr_trk_set_data_code", "gsdr_acq_read_profile_ex", "gsdr_stream_window_async", "gsdr_stream_release", "gsdr_stream_device",
    "gsdr_acq_dump_grid_step_two", "gsdr_acq_read_profile_intervals", "gsdr_acq_set_wipeoff",
    "gsdr_acq_get_spectrum_reuse", "gsdr_trk_force_loss_of_lock", "gsdr_acq_set_local_code",
    "gsdr_acq_set_active_prns", "gsdr_acq_submit_stream", "gsdr_acq_collect", "gsdr_host_register",
    "gsdr_host_unregister", "gsdr_trk_submit_stream", "gsdr_trk_collect", "gsdr_stream_landed",
    "gsdr_stream_wait_landed",
]

WIPE_EXACT, WIPE_GENERIC, WIPE_AVX2 = 0, 1, 2
SIGNAL_GPS_1C = 0
SIGNAL_GAL_1B = 1
SIGNAL_BDS_B1 = 2
TRK_F_VALID_OUTPUT, TRK_F_LOSS_OF_LOCK, TRK_F_PLL_180, TRK_F_BIT_SYNC, TRK_F_OVERRUN, TRK_F_LOGGED = 1, 2, 4, 8, 16, 32

# include/gsdr.h gsdr_trk_conf / gsdr_trk_epoch (C layout)
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


# The tracking block's dump record (dll_pll_veml_tracking.cc:1403-1500, log_data):
# 108 packed bytes per logged call, in the reference's write order.
TRK_DUMP_DTYPE = np.dtype([
    ("abs_VE", "<f4"), ("abs_E", "<f4"), ("abs_P", "<f4"), ("abs_L", "<f4"), ("abs_VL", "<f4"),
    ("Prompt_I", "<f4"), ("Prompt_Q", "<f4"), ("PRN_start_sample_count", "<u8"), ("acc_carrier_phase_rad", "<f4"),
    ("carrier_doppler_hz", "<f4"), ("carrier_doppler_rate_hz", "<f4"), ("code_freq_chips", "<f4"),
    ("code_freq_rate_chips", "<f4"), ("carr_error_hz", "<f4"), ("carr_error_filt_hz", "<f4"),
    ("code_error_chips", "<f4"), ("code_error_filt_chips", "<f4"), ("CN0_SNV_dB_Hz", "<f4"),
    ("carrier_lock_test", "<f4"), ("aux1", "<f4"), ("aux2", "<f8"), ("PRN", "<u4"),
    ("acq_code_phase_samples", "<f4"), ("acq_carrier_doppler_hz", "<f4"), ("EVM", "<f4")])
assert TRK_DUMP_DTYPE.itemsize == 108


def trk_dump_records(recs, fs_in, prn, acq_code_phase_samples, acq_carrier_doppler_hz, veml=False,
                     track_pilot=False):
    """The dump records the reference writes for a channel's calls: one per record
    flagged TRK_F_LOGGED (host/tracking_dump.cc is the C++ writer of the same bytes).
    acq_code_phase_samples is d_acq_code_phase_samples after the pull-in (:1817-1828)."""
    r = recs[(recs["flags"] & TRK_F_LOGGED) != 0]
    out = np.zeros(len(r), TRK_DUMP_DTYPE)
    ip = 2 if veml else 1
    acc = r["log_accu"]
    out["abs_VE"] = acc[:, 0] if veml else 0.0
    out["abs_E"], out["abs_P"], out["abs_L"] = acc[:, 1], acc[:, 2], acc[:, 3]
    out["abs_VL"] = acc[:, 4] if veml else 0.0
    out["Prompt_I"] = r["data_prompt"][:, 0] if track_pilot else r["taps"][:, 2 * ip]
    out["Prompt_Q"] = r["data_prompt"][:, 1] if track_pilot else r["taps"][:, 2 * ip + 1]
    stamp = r["sample_counter"] + r["consumed"].astype(np.uint64)
    out["PRN_start_sample_count"] = stamp
    out["acc_carrier_phase_rad"] = r["acc_carrier_phase_rad"].astype(np.float32)
    out["carrier_doppler_hz"] = r["carrier_doppler_hz"].astype(np.float32)
    two_pi = 2.0 * 3.1415926535897932384626433832795
    out["carrier_doppler_rate_hz"] = (r["carrier_rate"].astype(np.float64) * fs_in * fs_in / two_pi).astype(np.float32)
    out["code_freq_chips"] = r["code_freq_chips"].astype(np.float32)
    out["code_freq_rate_chips"] = (r["code_rate"].astype(np.float64) * fs_in * fs_in).astype(np.float32)
    out["carr_error_hz"] = r["carr_phase_error_hz"]
    out["carr_error_filt_hz"] = r["carr_error_filt_hz"]
    out["code_error_chips"] = r["code_error_chips"]
    out["code_error_filt_chips"] = r["code_error_filt_chips"]
    out["CN0_SNV_dB_Hz"] = r["cn0_db_hz"].astype(np.float32)
    out["carrier_lock_test"] = r["carrier_lock_test"].astype(np.float32)
    out["aux1"] = r["rem_code_phase_samples"].astype(np.float32)
    out["aux2"] = stamp.astype(np.float64)
    out["PRN"] = prn
    out["acq_code_phase_samples"] = np.float32(acq_code_phase_samples)
    out["acq_carrier_doppler_hz"] = np.float32(acq_carrier_doppler_hz)
    out["EVM"] = r["evm"].astype(np.float32)
    return out


def read_trk_dump(path):
    """A tracking dump file (the reference's trk_channel_<n>.dat layout) as records."""
    return np.fromfile(path, dtype=TRK_DUMP_DTYPE)


class GsdrError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("gsdr error %d: %s" % (code, msg))
        self.code = code


class AcqConf(ctypes.Structure):
    _fields_ = [
        ("fs_in", ctypes.c_int64),
        ("consumed_samples", ctypes.c_uint32),
        ("fft_size", ctypes.c_uint32),
        ("samples_per_code", ctypes.c_float),
        ("samples_per_chip", ctypes.c_uint32),
        ("doppler_max", ctypes.c_int32),
        ("doppler_step", ctypes.c_uint32),
        ("doppler_center", ctypes.c_int32),
        ("doppler_bias", ctypes.c_int32),
        ("num_doppler_bins", ctypes.c_uint32),
        ("pfa", ctypes.c_float),
        ("max_dwells", ctypes.c_uint32),
        ("bit_transition_flag", ctypes.c_int32),
        ("item_type", ctypes.c_int32),
        ("max_prns", ctypes.c_uint32),
        ("max_blocks", ctypes.c_uint32),
        ("sampled_ms", ctypes.c_uint32),
        ("ms_per_code", ctypes.c_uint32),
    ]


class AcqResult(ctypes.Structure):
    _fields_ = [
        ("prn", ctypes.c_uint32),
        ("doppler_index", ctypes.c_uint32),
        ("code_phase", ctypes.c_uint32),
        ("doppler_hz", ctypes.c_int32),
        ("peak", ctypes.c_float),
        ("input_power", ctypes.c_float),
        ("second_peak", ctypes.c_float),
        ("test_statistic", ctypes.c_float),
        ("acq_delay_samples", ctypes.c_double),
        ("samplestamp", ctypes.c_uint64),
        ("positive", ctypes.c_int32),
        ("num_dwells", ctypes.c_int32),
    ]


ACQ_RESULT_DTYPE = np.dtype([
    ("prn", np.uint32), ("doppler_index", np.uint32), ("code_phase", np.uint32), ("doppler_hz", np.int32),
    ("peak", np.float32), ("input_power", np.float32), ("second_peak", np.float32),
    ("test_statistic", np.float32), ("acq_delay_samples", np.float64), ("samplestamp", np.uint64),
    ("positive", np.int32), ("num_dwells", np.int32)])
assert ACQ_RESULT_DTYPE.itemsize == ctypes.sizeof(AcqResult)


class CorrJob(ctypes.Structure):
    _fields_ = [
        ("channel", ctypes.c_int32),
        ("n_samples", ctypes.c_int32),
        ("sample_offset", ctypes.c_int64),
        ("rem_carr_phase_rad", ctypes.c_float),
        ("carr_phase_step_rad", ctypes.c_float),
        ("carr_phase_rate_step_rad", ctypes.c_float),
        ("rem_code_phase_chips", ctypes.c_float),
        ("code_phase_step_chips", ctypes.c_float),
        ("code_phase_rate_step_chips", ctypes.c_float),
    ]


CORR_JOB_DTYPE = np.dtype([
    ("channel", np.int32), ("n_samples", np.int32), ("sample_offset", np.int64),
    ("rem_carr_phase_rad", np.float32), ("carr_phase_step_rad", np.float32),
    ("carr_phase_rate_step_rad", np.float32), ("rem_code_phase_chips", np.float32),
    ("code_phase_step_chips", np.float32), ("code_phase_rate_step_chips", np.float32)])
assert CORR_JOB_DTYPE.itemsize == ctypes.sizeof(CorrJob)

_lib = None


def load():
    """Load libgsdr.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError("libgsdr.so not built: %s (run __graft_entry__.build())" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    P, I, U32, U64, I64, F = (ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64,
                              ctypes.c_float)
    L.gsdr_last_error.restype = ctypes.c_char_p
    L.gsdr_abi_version.restype = I
    L.gsdr_device_count.argtypes = [P]
    L.gsdr_acq_create.argtypes = [I, ctypes.POINTER(AcqConf), P]
    L.gsdr_acq_destroy.argtypes = [P]
    L.gsdr_acq_destroy.restype = None
    L.gsdr_acq_get_dims.argtypes = [P, P, P]
    L.gsdr_acq_set_local_codes.argtypes = [P, P, P, U32]
    L.gsdr_acq_set_doppler.argtypes = [P, ctypes.c_int32, U32, ctypes.c_int32]
    L.gsdr_acq_set_threshold.argtypes = [P, F]
    L.gsdr_acq_get_threshold.argtypes = [P, P]
    L.gsdr_acq_run.argtypes = [P, P, U32, U64, P]
    L.gsdr_acq_run_device.argtypes = [P, P, U32, U64, U64, P, P]
    L.gsdr_acq_dump_grid.argtypes = [P, P, U32, P]
    L.gsdr_acq_dump_grid_step_two.argtypes = [P, P, U32, ctypes.c_float, P]
    L.gsdr_acq_read_profile_intervals.argtypes = [P, P, ctypes.c_int, P, P, U32, P]
    L.gsdr_acq_set_wipeoff.argtypes = [P, ctypes.c_int]
    L.gsdr_acq_get_spectrum_reuse.argtypes = [P, P, P]
    L.gsdr_acq_dump_spectra.argtypes = [P, P, P]
    L.gsdr_corr_create.argtypes = [I, I, I, I, P]
    L.gsdr_corr_destroy.argtypes = [P]
    L.gsdr_corr_destroy.restype = None
    L.gsdr_corr_set_local_code_and_taps.argtypes = [P, I, I, P, P, I]
    L.gsdr_corr_set_local_code_and_taps_complex.argtypes = [P, I, I, P, P, I]
    L.gsdr_corr_set_high_dynamics_resampler.argtypes = [P, I, I]
    L.gsdr_corr_set_resampler_assoc.argtypes = [P, I]
    L.gsdr_corr_run.argtypes = [P, I, P, I, F, F, F, F, F, F, I, P]
    L.gsdr_corr_run_batch.argtypes = [P, P, I, P, I, I64, P, P]
    L.gsdr_corr_run_batch_device.argtypes = [P, P, I, P, I, I64, P, P]
    L.gsdr_corr_dump_indices.argtypes = [P, I, F, F, I, P]
    L.gsdr_acq_set_profiling.argtypes = [P, I]
    L.gsdr_acq_read_profile.argtypes = [P, P, P]
    L.gsdr_corr_run_epochs.argtypes = [P, P, I, I, P, I, I64, P, P]
    L.gsdr_corr_set_profiling.argtypes = [P, I]
    L.gsdr_corr_read_profile.argtypes = [P, P, P]
    L.gsdr_trk_conf_default.argtypes = [P]
    L.gsdr_trk_conf_default.restype = None
    L.gsdr_trk_create.argtypes = [I, P, P]
    L.gsdr_trk_destroy.argtypes = [P]
    L.gsdr_trk_destroy.restype = None
    L.gsdr_trk_start.argtypes = [P, I, U32, P, I, ctypes.c_double, ctypes.c_double, U64, U64, P]
    L.gsdr_trk_stop.argtypes = [P, I]
    L.gsdr_trk_force_loss_of_lock.argtypes = [P, I]
    L.gsdr_acq_set_local_code.argtypes = [P, U32, P, U32]
    L.gsdr_acq_set_active_prns.argtypes = [P, U32]
    L.gsdr_acq_submit_stream.argtypes = [P, P, U64, U32, U64]
    L.gsdr_acq_collect.argtypes = [P, P, P, P]
    L.gsdr_host_register.argtypes = [P, ctypes.c_size_t]
    L.gsdr_host_unregister.argtypes = [P]
    L.gsdr_trk_set_data_code.argtypes = [P, I, P, I]
    L.gsdr_trk_run_device.argtypes = [P, P, U64, U64, U32, P, P, P]
    L.gsdr_trk_run.argtypes = [P, P, U64, U64, U32, P, P]
    L.gsdr_trk_get_channel.argtypes = [P, I, P, P, P, P]
    L.gsdr_trk_save_state.argtypes = [P, I, P]
    L.gsdr_trk_restore_state.argtypes = [P, I, P]
    L.gsdr_trk_set_profiling.argtypes = [P, I]
    L.gsdr_trk_read_profile.argtypes = [P, P, P]
    L.gsdr_acq_set_cu_mask.argtypes = [P, P, I]
    L.gsdr_acq_set_step_two.argtypes = [P, U32, F, F]
    L.gsdr_acq_get_step_two_threshold.argtypes = [P, P]
    L.gsdr_acq_run_step_two.argtypes = [P, P, U32, P, P, P, U64, P]
    L.gsdr_trk_set_cu_mask.argtypes = [P, P, I]
    L.gsdr_acq_run_dwell.argtypes = [P, P, U32, U64, P]
    L.gsdr_stream_create.argtypes = [I, I, U64, U64, P]
    L.gsdr_stream_destroy.argtypes = [P]
    L.gsdr_stream_destroy.restype = None
    L.gsdr_stream_push.argtypes = [P, P, U64, U64]
    L.gsdr_stream_landed.argtypes = [P, P]
    L.gsdr_stream_wait_landed.argtypes = [P, U64]
    L.gsdr_stream_span.argtypes = [P, P, P]
    L.gsdr_stream_window.argtypes = [P, U64, U64, P]
    L.gsdr_acq_read_profile_ex.argtypes = [P, P, P, P]
    L.gsdr_stream_window_async.argtypes = [P, U64, U64, P, P]
    L.gsdr_stream_release.argtypes = [P, P]
    L.gsdr_stream_device.argtypes = [P, P]
    L.gsdr_acq_run_stream.argtypes = [P, P, U64, U32, U64, P]
    L.gsdr_trk_run_stream.argtypes = [P, P, U32, P, P, P]
    L.gsdr_trk_run_stream_host.argtypes = [P, P, U32, P, P]
    L.gsdr_trk_submit_stream.argtypes = [P, P, U32]
    L.gsdr_trk_collect.argtypes = [P, ctypes.c_int, P, P, P]
    _lib = L
    return L


def _check(rc):
    if rc != GSDR_OK:
        raise GsdrError(rc, load().gsdr_last_error().decode(errors="replace"))


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def device_count():
    n = ctypes.c_int(0)
    _check(load().gsdr_device_count(ctypes.byref(n)))
    return n.value


class Acquisition:
    """Batched PCPS acquisition (pcps_acquisition equivalent) on one GPU."""

    def __init__(self, fs_in, consumed_samples, doppler_max, doppler_step, pfa=0.0, max_prns=32, max_blocks=1,
                 samples_per_code=None, samples_per_chip=None, num_doppler_bins=0, doppler_center=0,
                 doppler_bias=0, item_type=ITEM_GR_COMPLEX, fft_size=0, sampled_ms=1, ms_per_code=1,
                 chip_rate=1023000.0, max_dwells=1, bit_transition=False, device=0):
        L = load()
        c = AcqConf()
        c.fs_in = int(fs_in)
        c.consumed_samples = int(consumed_samples)
        c.fft_size = int(fft_size)
        spms = np.float32(np.float32(fs_in) * np.float32(0.001))
        c.samples_per_code = float(samples_per_code if samples_per_code is not None else spms * ms_per_code)
        c.samples_per_chip = int(samples_per_chip if samples_per_chip is not None
                                 else int(np.ceil(float(np.float32(fs_in)) / chip_rate)))
        c.doppler_max = int(doppler_max)
        c.doppler_step = int(doppler_step)
        c.doppler_center = int(doppler_center)
        c.doppler_bias = int(doppler_bias)
        c.num_doppler_bins = int(num_doppler_bins)
        c.pfa = float(pfa)
        c.max_dwells = int(max_dwells)
        c.bit_transition_flag = int(bool(bit_transition))
        c.item_type = int(item_type)
        c.max_prns = int(max_prns)
        c.max_blocks = int(max_blocks)
        c.sampled_ms = int(sampled_ms)
        c.ms_per_code = int(ms_per_code)
        self.conf = c
        self._h = ctypes.c_void_p()
        _check(L.gsdr_acq_create(int(device), ctypes.byref(c), ctypes.byref(self._h)))
        D, N = ctypes.c_uint32(), ctypes.c_uint32()
        _check(L.gsdr_acq_get_dims(self._h, ctypes.byref(D), ctypes.byref(N)))
        self.num_doppler_bins, self.fft_size = D.value, N.value
        self.nprn = 0
        self.item_type = item_type
        self.dwells = 1 if bit_transition else max(1, int(max_dwells))

    def close(self):
        if self._h:
            load().gsdr_acq_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_local_codes(self, codes, prns):
        codes = np.ascontiguousarray(codes, np.complex64)
        prns = np.ascontiguousarray(prns, np.uint32)
        assert codes.ndim == 2 and codes.shape[0] == len(prns)
        _check(load().gsdr_acq_set_local_codes(self._h, _ptr(codes), _ptr(prns), len(prns)))
        self.nprn = len(prns)

    def set_doppler(self, doppler_max, doppler_step, doppler_center=0):
        _check(load().gsdr_acq_set_doppler(self._h, int(doppler_max), int(doppler_step), int(doppler_center)))

    def set_wipeoff(self, mode):
        """Carrier model of the Doppler grid: WIPE_EXACT (default), WIPE_GENERIC, WIPE_AVX2
        (include/gsdr.h gsdr_acq_set_wipeoff); accepts the names too."""
        if isinstance(mode, str):
            mode = {"exact": WIPE_EXACT, "generic": WIPE_GENERIC, "avx2": WIPE_AVX2}[mode]
        _check(load().gsdr_acq_set_wipeoff(self._h, int(mode)))
        self._wipe_mode = int(mode)

    @property
    def wipe_mode(self):
        """The carrier model in effect (the handle starts from GSDR_ACQ_WIPE, else exact)."""
        if getattr(self, "_wipe_mode", None) is None:
            env = os.environ.get("GSDR_ACQ_WIPE", "exact")
            self._wipe_mode = {"generic": WIPE_GENERIC, "avx2": WIPE_AVX2}.get(env, WIPE_EXACT)
        return self._wipe_mode

    @property
    def spectrum_reuse(self):
        """(q, p): q forward spectra per block (== D: none), p bins of shift per class step."""
        q = np.zeros(1, np.uint32)
        p = np.zeros(1, np.uint32)
        _check(load().gsdr_acq_get_spectrum_reuse(self._h, _ptr(q), _ptr(p)))
        return int(q[0]), int(p[0])

    def set_threshold(self, t):
        _check(load().gsdr_acq_set_threshold(self._h, float(t)))

    @property
    def threshold(self):
        t = ctypes.c_float()
        _check(load().gsdr_acq_get_threshold(self._h, ctypes.byref(t)))
        return t.value

    def _items(self, iq):
        return np.ascontiguousarray(iq, _ITEM_NP[int(self.item_type)])

    def run(self, iq, nblocks=1, stamp0=0):
        """Synchronous drop-in: host IQ of nblocks*max_dwells*consumed items (nblocks
        attempts of max_dwells blocks) -> structured array [nblocks, nprn]."""
        iq = self._items(iq)
        out = np.zeros(nblocks * self.nprn, ACQ_RESULT_DTYPE)
        _check(load().gsdr_acq_run(self._h, _ptr(iq), int(nblocks), int(stamp0), _ptr(out)))
        return out.reshape(nblocks, self.nprn)

    def run_dwell(self, iq, dwell, stamp=0):
        """acquisition_core's per-call dwell (gsdr_acq_run_dwell): one block of host
        IQ added to the device grid of the attempt (dwell 0 starts it) ->
        structured array [nprn]."""
        iq = self._items(iq)
        out = np.zeros(self.nprn, ACQ_RESULT_DTYPE)
        _check(load().gsdr_acq_run_dwell(self._h, _ptr(iq), int(dwell), int(stamp), _ptr(out)))
        return out

    def run_stream(self, ring, first_sample, nblocks=1, stamp0=0):
        """nblocks attempts read in place from a Stream (device IQ ring) from
        absolute sample first_sample -> structured array [nblocks, nprn]."""
        out = np.zeros(nblocks * self.nprn, ACQ_RESULT_DTYPE)
        _check(load().gsdr_acq_run_stream(self._h, ring._h, int(first_sample), int(nblocks), int(stamp0), _ptr(out)))
        return out.reshape(nblocks, self.nprn)

    def set_step_two(self, num_doppler_bins_step2=4, doppler_step2=125.0, pfa2=0.0):
        """make_two_steps narrow grid (Acq_Conf second_nbins / second_doppler_step /
        pfa_second_step; pcps_acquisition.cc:298-314, :717-773)."""
        _check(load().gsdr_acq_set_step_two(self._h, int(num_doppler_bins_step2), float(doppler_step2),
                                            float(pfa2)))
        self._st2_bins = int(num_doppler_bins_step2)

    @property
    def step_two_threshold(self):
        t = ctypes.c_float()
        _check(load().gsdr_acq_get_step_two_threshold(self._h, ctypes.byref(t)))
        return t.value

    def run_step_two(self, iq, prn_slots, doppler_centers_hz, coarse_input_power, stamp=0):
        """Second step for the given PRN slots on one attempt of host IQ, centred on
        each slot's coarse Acq_doppler_hz -> structured array [len(prn_slots)]."""
        iq = self._items(iq)
        slots = np.ascontiguousarray(prn_slots, np.uint32)
        cen = np.ascontiguousarray(doppler_centers_hz, np.float32)
        ip = np.ascontiguousarray(coarse_input_power, np.float32)
        assert len(slots) == len(cen) == len(ip)
        out = np.zeros(len(slots), ACQ_RESULT_DTYPE)
        _check(load().gsdr_acq_run_step_two(self._h, _ptr(iq), len(slots), _ptr(slots), _ptr(cen), _ptr(ip),
                                            int(stamp), _ptr(out)))
        return out

    def run_device(self, iq_dev_ptr, nblocks, stride_items, stamp0, out_dev_ptr, stream_ptr=0):
        _check(load().gsdr_acq_run_device(self._h, ctypes.c_void_p(iq_dev_ptr), int(nblocks), int(stride_items),
                                          int(stamp0), ctypes.c_void_p(out_dev_ptr), ctypes.c_void_p(stream_ptr)))

    def set_profiling(self, enable):
        _check(load().gsdr_acq_set_profiling(self._h, int(bool(enable))))

    def set_cu_mask(self, mask_words):
        m = np.ascontiguousarray(mask_words, np.uint32)
        _check(load().gsdr_acq_set_cu_mask(self._h, _ptr(m) if len(m) else None, len(m)))

    def read_profile(self):
        """(stage_ms[4], launches[4]): forward, correlate, reduce, second peak."""
        ms = np.zeros(4, np.float64)
        n = np.zeros(4, np.uint32)
        _check(load().gsdr_acq_read_profile(self._h, _ptr(ms), _ptr(n)))
        return ms, n

    def read_profile_ex(self):
        """(stage_ms[4], launches[4], busy_ms[4]): busy = union of the stage's launch intervals."""
        ms = np.zeros(4, np.float64)
        n = np.zeros(4, np.uint32)
        busy = np.zeros(4, np.float64)
        _check(load().gsdr_acq_read_profile_ex(self._h, _ptr(ms), _ptr(n), _ptr(busy)))
        return ms, n, busy

    def read_profile_intervals(self, ref_event, stage, max_n=4096):
        """[start, end) ms of each recorded launch of `stage` against ref_event (a
        hipEvent_t handle, e.g. torch.cuda.Event(enable_timing=True).cuda_event)."""
        st = np.zeros(max_n, np.float64)
        en = np.zeros(max_n, np.float64)
        n = ctypes.c_uint32(0)
        _check(load().gsdr_acq_read_profile_intervals(self._h, ctypes.c_void_p(ref_event), int(stage), _ptr(st),
                                                      _ptr(en), int(max_n), ctypes.byref(n)))
        k = min(n.value, max_n)
        return st[:k], en[:k]

    def dump_grid(self, iq, prn_slot):
        iq = self._items(iq)
        g = np.zeros((self.num_doppler_bins, self.fft_size), np.float32)
        _check(load().gsdr_acq_dump_grid(self._h, _ptr(iq), int(prn_slot), _ptr(g)))
        return g

    def dump_grid_step_two(self, iq, prn_slot, doppler_center_hz):
        """The make_two_steps narrow grid of one block (set_step_two first)."""
        iq = self._items(iq)
        g = np.zeros((self._st2_bins, self.fft_size), np.float32)
        _check(load().gsdr_acq_dump_grid_step_two(self._h, _ptr(iq), int(prn_slot), float(doppler_center_hz), _ptr(g)))
        return g

    def dump_spectra(self, iq):
        iq = self._items(iq)
        X = np.zeros((self.num_doppler_bins, self.fft_size), np.complex64)
        _check(load().gsdr_acq_dump_spectra(self._h, _ptr(iq), _ptr(X)))
        return X


class Correlator:
    """Batched tracking multicorrelator (Cpu_Multicorrelator_Real_Codes equivalent)."""

    def __init__(self, max_channels, max_len, max_taps=8, device=0):
        self._h = ctypes.c_void_p()
        _check(load().gsdr_corr_create(int(device), int(max_channels), int(max_len), int(max_taps),
                                       ctypes.byref(self._h)))
        self.max_taps = max_taps
        self.ntaps = {}

    def close(self):
        if self._h:
            load().gsdr_corr_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_local_code_and_taps(self, channel, code, shifts):
        if np.iscomplexobj(code):
            code = np.ascontiguousarray(code, np.complex64)
            shifts = np.ascontiguousarray(shifts, np.float32)
            _check(load().gsdr_corr_set_local_code_and_taps_complex(self._h, channel, len(code), _ptr(code),
                                                                    _ptr(shifts), len(shifts)))
        else:
            code = np.ascontiguousarray(code, np.float32)
            shifts = np.ascontiguousarray(shifts, np.float32)
            _check(load().gsdr_corr_set_local_code_and_taps(self._h, channel, len(code), _ptr(code), _ptr(shifts),
                                                            len(shifts)))
        self.ntaps[channel] = len(shifts)

    def set_high_dynamics_resampler(self, channel, enable):
        _check(load().gsdr_corr_set_high_dynamics_resampler(self._h, channel, int(bool(enable))))

    def set_resampler_assoc(self, assoc):
        _check(load().gsdr_corr_set_resampler_assoc(self._h, int(assoc)))

    def run(self, channel, sig, rem_carr, carr_step, rem_code, code_step, n, carr_rate=0.0, code_rate=0.0,
            item_type=ITEM_GR_COMPLEX):
        """Carrier_wipeoff_multicorrelator_resampler (7-argument form), synchronous."""
        sig = np.ascontiguousarray(sig, _ITEM_NP[int(item_type)])
        out = np.zeros(self.ntaps[channel], np.complex64)
        _check(load().gsdr_corr_run(self._h, channel, _ptr(sig), item_type, rem_carr, carr_step, carr_rate, rem_code,
                                    code_step, code_rate, int(n), _ptr(out)))
        return out

    def run_batch(self, jobs, iq_dev_ptr, iq_items, out_dev_ptr, item_type=ITEM_GR_COMPLEX, stream_ptr=0):
        jobs = np.ascontiguousarray(jobs, CORR_JOB_DTYPE)
        _check(load().gsdr_corr_run_batch(self._h, _ptr(jobs), len(jobs), ctypes.c_void_p(iq_dev_ptr), item_type,
                                          int(iq_items), ctypes.c_void_p(out_dev_ptr), ctypes.c_void_p(stream_ptr)))

    def run_batch_device(self, jobs_dev_ptr, njobs, iq_dev_ptr, iq_items, out_dev_ptr, item_type=ITEM_GR_COMPLEX,
                         stream_ptr=0):
        _check(load().gsdr_corr_run_batch_device(self._h, ctypes.c_void_p(jobs_dev_ptr), int(njobs),
                                                 ctypes.c_void_p(iq_dev_ptr), item_type, int(iq_items),
                                                 ctypes.c_void_p(out_dev_ptr), ctypes.c_void_p(stream_ptr)))

    def run_epochs(self, jobs_dev_ptr, jobs_per_epoch, n_epochs, iq_dev_ptr, iq_items, out_dev_ptr,
                   item_type=ITEM_GR_COMPLEX, stream_ptr=0):
        _check(load().gsdr_corr_run_epochs(self._h, ctypes.c_void_p(jobs_dev_ptr), int(jobs_per_epoch), int(n_epochs),
                                           ctypes.c_void_p(iq_dev_ptr), item_type, int(iq_items),
                                           ctypes.c_void_p(out_dev_ptr), ctypes.c_void_p(stream_ptr)))

    def set_profiling(self, enable):
        _check(load().gsdr_corr_set_profiling(self._h, int(bool(enable))))

    def read_profile(self):
        ms = ctypes.c_double()
        n = ctypes.c_uint32()
        _check(load().gsdr_corr_read_profile(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def dump_indices(self, channel, rem_code, code_step, n):
        out = np.zeros((self.ntaps[channel], n), np.int32)
        _check(load().gsdr_corr_dump_indices(self._h, channel, rem_code, code_step, int(n), _ptr(out)))
        return out


def trk_conf_default():
    """Dll_Pll_Conf defaults (gsdr_trk_conf_default) as a one-element structured array."""
    c = np.zeros(1, TRK_CONF_DTYPE)
    load().gsdr_trk_conf_default(_ptr(c))
    return c


class Tracking:
    """Device-resident DLL/PLL tracking (dll_pll_veml_tracking) for a pool of channels."""

    def __init__(self, conf, device=0):
        self.conf = np.ascontiguousarray(conf, TRK_CONF_DTYPE).copy()
        self._h = ctypes.c_void_p()
        _check(load().gsdr_trk_create(int(device), _ptr(self.conf), ctypes.byref(self._h)))
        self.max_channels = int(self.conf["max_channels"][0])

    def close(self):
        if self._h:
            load().gsdr_trk_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def start(self, ch, prn, code, acq_delay_samples, acq_doppler_hz, acq_samplestamp, nitems_read, data_code=None):
        """start_tracking + the state-1 pull-in call; data_code: the data component's
        replica for pilot tracking (Galileo E1 with track_pilot)."""
        code = np.ascontiguousarray(code, np.float32)
        if data_code is not None:
            dc = np.ascontiguousarray(data_code, np.float32)
            _check(load().gsdr_trk_set_data_code(self._h, int(ch), _ptr(dc), len(dc)))
        first = ctypes.c_uint64()
        _check(load().gsdr_trk_start(self._h, int(ch), int(prn), _ptr(code), len(code), float(acq_delay_samples),
                                     float(acq_doppler_hz), int(acq_samplestamp), int(nitems_read),
                                     ctypes.byref(first)))
        return first.value

    def stop(self, ch):
        _check(load().gsdr_trk_stop(self._h, int(ch)))

    def force_loss_of_lock(self, ch):
        """A telemetry fault for channel ch (msg_handler_telemetry_to_trk,
        dll_pll_veml_tracking.cc:614-637): its next lock check reports loss of lock."""
        _check(load().gsdr_trk_force_loss_of_lock(self._h, int(ch)))

    def run(self, iq, iq_first_sample, max_epochs):
        """Synchronous: host IQ -> (records [max_channels, max_epochs], counts [max_channels])."""
        item = int(self.conf["item_type"][0])
        iq = np.ascontiguousarray(iq, _ITEM_NP[item])
        n_items = len(iq) if item == ITEM_GR_COMPLEX else len(iq) // 2
        out = np.zeros(self.max_channels * max_epochs, TRK_EPOCH_DTYPE)
        n = np.zeros(self.max_channels, np.uint32)
        _check(load().gsdr_trk_run(self._h, _ptr(iq), int(iq_first_sample), int(n_items), int(max_epochs), _ptr(out),
                                   _ptr(n)))
        return out.reshape(self.max_channels, max_epochs), n

    def run_device(self, iq_dev_ptr, iq_first_sample, iq_items, max_epochs, out_dev_ptr, nout_dev_ptr, stream_ptr=0):
        _check(load().gsdr_trk_run_device(self._h, ctypes.c_void_p(iq_dev_ptr), int(iq_first_sample), int(iq_items),
                                          int(max_epochs), ctypes.c_void_p(out_dev_ptr), ctypes.c_void_p(nout_dev_ptr),
                                          ctypes.c_void_p(stream_ptr)))

    def run_stream(self, ring, max_epochs, out_dev_ptr, nout_dev_ptr, stream_ptr=0):
        """Advance the channels over a Stream's newest contiguous window
        (gsdr_trk_run_stream); asynchronous."""
        _check(load().gsdr_trk_run_stream(self._h, ring._h, int(max_epochs), ctypes.c_void_p(out_dev_ptr),
                                          ctypes.c_void_p(nout_dev_ptr), ctypes.c_void_p(stream_ptr)))

    def run_stream_host(self, ring, max_epochs):
        """gsdr_trk_run_stream_host: synchronous ring form -> (records, counts) on the host."""
        out = np.zeros(self.max_channels * max_epochs, TRK_EPOCH_DTYPE)
        n = np.zeros(self.max_channels, np.uint32)
        _check(load().gsdr_trk_run_stream_host(self._h, ring._h, int(max_epochs), _ptr(out), _ptr(n)))
        return out.reshape(self.max_channels, max_epochs), n

    def submit_stream(self, ring, max_epochs):
        """gsdr_trk_submit_stream: the ring form with the records copied back behind it; no wait
        (up to two submissions in flight)."""
        _check(load().gsdr_trk_submit_stream(self._h, ring._h, int(max_epochs)))
        self._sub_epochs = getattr(self, "_sub_epochs", [])
        self._sub_epochs.append(int(max_epochs))

    def collect(self, wait=True):
        """gsdr_trk_collect -> (records, counts) of the oldest submission, or None while it is in
        flight (wait=False)."""
        pending = getattr(self, "_sub_epochs", [])
        me = pending[0] if pending else 1
        out = np.zeros(self.max_channels * me, TRK_EPOCH_DTYPE)
        n = np.zeros(self.max_channels, np.uint32)
        got = ctypes.c_uint32()
        rc = load().gsdr_trk_collect(self._h, 1 if wait else 0, _ptr(out), _ptr(n), ctypes.byref(got))
        if rc == 1:
            return None
        _check(rc)
        pending.pop(0)
        return out.reshape(self.max_channels, me), n

    def channel(self, ch):
        st, nxt, dop, cn0 = ctypes.c_int32(), ctypes.c_uint64(), ctypes.c_double(), ctypes.c_double()
        _check(load().gsdr_trk_get_channel(self._h, int(ch), ctypes.byref(st), ctypes.byref(nxt), ctypes.byref(dop),
                                           ctypes.byref(cn0)))
        return {"state": st.value, "next_sample": nxt.value, "carrier_doppler_hz": dop.value, "cn0_db_hz": cn0.value}

    def save_state(self, slot=0, stream_ptr=0):
        _check(load().gsdr_trk_save_state(self._h, int(slot), ctypes.c_void_p(stream_ptr)))

    def restore_state(self, slot=0, stream_ptr=0):
        _check(load().gsdr_trk_restore_state(self._h, int(slot), ctypes.c_void_p(stream_ptr)))

    def set_profiling(self, enable):
        _check(load().gsdr_trk_set_profiling(self._h, int(bool(enable))))

    def set_cu_mask(self, mask_words):
        m = np.ascontiguousarray(mask_words, np.uint32)
        _check(load().gsdr_trk_set_cu_mask(self._h, _ptr(m) if len(m) else None, len(m)))

    def read_profile(self):
        ms = ctypes.c_double()
        n = ctypes.c_uint32()
        _check(load().gsdr_trk_read_profile(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value


class Stream:
    """Device IQ ring indexed by absolute sample count (gsdr_stream_*): push the
    input stream once, read it in place from Acquisition.run_stream and
    Tracking.run_stream."""

    def __init__(self, item_type, capacity_items, max_window_items, device=0):
        self._h = ctypes.c_void_p()
        _check(load().gsdr_stream_create(int(device), int(item_type), int(capacity_items), int(max_window_items),
                                         ctypes.byref(self._h)))
        self.item_type = int(item_type)
        self._inflight = []  # (end, array) of pushes whose copies may still read the array

    def close(self):
        if self._h:
            load().gsdr_stream_destroy(self._h)
            self._h = ctypes.c_void_p()
        self._inflight = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push(self, iq, first_sample):
        """Asynchronous push (gsdr_stream_push): the array (or the contiguous copy made
        of it here) is held until its copy landed; the caller's own array must not be
        modified before landed() >= first_sample + n (or wait_landed)."""
        iq = np.ascontiguousarray(iq, _ITEM_NP[self.item_type])
        n = len(iq) if self.item_type == ITEM_GR_COMPLEX else len(iq) // 2
        _check(load().gsdr_stream_push(self._h, _ptr(iq), int(first_sample), int(n)))
        self._inflight.append((int(first_sample) + n, iq))
        self.landed()
        return n

    def landed(self):
        """Every item before the returned index is in device memory (gsdr_stream_landed)."""
        v = ctypes.c_uint64()
        _check(load().gsdr_stream_landed(self._h, ctypes.byref(v)))
        self._inflight = [(e, a) for e, a in self._inflight if e > v.value]
        return v.value

    def wait_landed(self, upto):
        _check(load().gsdr_stream_wait_landed(self._h, int(upto)))
        return self.landed()

    def span(self):
        f, n = ctypes.c_uint64(), ctypes.c_uint64()
        _check(load().gsdr_stream_span(self._h, ctypes.byref(f), ctypes.byref(n)))
        return f.value, n.value

    def window(self, first_sample, n_items):
        p = ctypes.c_void_p()
        _check(load().gsdr_stream_window(self._h, int(first_sample), int(n_items), ctypes.byref(p)))
        return p.value

    def window_async(self, first_sample, n_items, consumer_stream):
        """Window for reads enqueued on consumer_stream (a hipStream_t handle, e.g.
        torch.cuda.Stream.cuda_stream); call release(consumer_stream) after them."""
        p = ctypes.c_void_p()
        _check(load().gsdr_stream_window_async(self._h, int(first_sample), int(n_items),
                                               ctypes.c_void_p(consumer_stream), ctypes.byref(p)))
        return p.value

    def release(self, consumer_stream):
        _check(load().gsdr_stream_release(self._h, ctypes.c_void_p(consumer_stream)))

    @contextlib.contextmanager
    def reading(self, first_sample, n_items, consumer_stream):
        """window_async .. release as a context: the window is released (the
        reads enqueued so far covered) even when the consumer's code raises, so a
        later push never waits on a window nobody will close."""
        p = self.window_async(first_sample, n_items, consumer_stream)
        try:
            yield p
        finally:
            self.release(consumer_stream)

    @property
    def device(self):
        d = ctypes.c_int()
        _check(load().gsdr_stream_device(self._h, ctypes.byref(d)))
        return d.value


def cu_partition(n_reserved, n_cus=256):
    """CU masks (hipExtStreamCreateWithCUMask numbering: bit i = CU i//8 of XCD i%8)
    giving the first n_reserved CUs, spread over the 8 XCDs, to one stream and the
    rest to another.  Returns (reserved_mask, rest_mask) as uint32 word arrays."""
    words = (n_cus + 31) // 32
    res = np.zeros(words, np.uint32)
    for i in range(n_reserved):
        res[i // 32] |= np.uint32(1 << (i % 32))
    full = np.full(words, 0xFFFFFFFF, np.uint32)
    return res, full & ~res
