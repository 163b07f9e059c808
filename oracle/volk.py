"""ORACLE — test infrastructure only.  ctypes front-end of oracle/volk_oracle.c.

Builds oracle/build/liboracle.so on first use if it is missing (gcc; no GPU).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_f = ctypes.c_float
_u = ctypes.c_uint
_i = ctypes.c_int
_p = ctypes.c_void_p


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(_HERE, f) for f in ("volk_oracle.c", "trk_oracle.c")]
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < max(os.path.getmtime(f) for f in srcs):
            build()
        L = ctypes.CDLL(_SO)
        L.orc_resampler_32f_xn.argtypes = [_p, _p, _f, _f, _p, _u, _i, _u, _i]
        L.orc_resampler_index.argtypes = [_p, _f, _f, _p, _u, _i, _u, _i]
        L.orc_resampler_32fc_xn.argtypes = [_p, _p, _f, _f, _p, _u, _i, _u, _i]
        L.orc_high_dyn_resampler_32f_xn.argtypes = [_p, _p, _f, _f, _f, _p, _u, _i, _u]
        L.orc_rotator_dot_prod_32fc_32f_xn.argtypes = [_p, _p, _f, _f, _p, _p, _i, _u]
        L.orc_rotator_dot_prod_32fc_32f_xn_avx.argtypes = [_p, _p, _f, _f, _p, _p, _i, _u]
        L.orc_multicorrelator_real_codes_avx.argtypes = [_p, _p, _p, _u, _p, _i, _f, _f, _f, _f, _u]
        L.orc_rotator_dot_prod_32fc_x2_xn.argtypes = [_p, _p, _f, _f, _p, _p, _i, _u]
        L.orc_high_dyn_rotator_dot_prod_32fc_32f_xn.argtypes = [_p, _p, _f, _f, _f, _f, _p, _p, _i, _u]
        L.orc_s32f_sincos_32fc.argtypes = [_p, _f, _p, _u]
        L.orc_s32f_sincos_32fc_avx2.argtypes = [_p, _f, _p, _u]
        L.orc_index_max_32u.argtypes = [_p, ctypes.c_uint32]
        L.orc_index_max_32u.restype = ctypes.c_uint32
        L.orc_multicorrelator_real_codes.argtypes = [_p, _p, _p, _u, _p, _i, _f, _f, _f, _f, _f, _f, _u, _i, _i]
        L.orc_multicorrelator_complex_codes.argtypes = [_p, _p, _p, _u, _p, _i, _f, _f, _f, _f, _u, _i]
        L.orc_multicorrelator_real_codes_exact.argtypes = [_p, _p, _p, _u, _p, _i, _f, _f, _f, _f, _u, _i]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def resampler_index(rem, step, shifts, L, N, assoc=1):
    shifts = _c(shifts, np.float32)
    out = np.empty((len(shifts), N), np.int32)
    lib().orc_resampler_index(_ptr(out), rem, step, _ptr(shifts), L, len(shifts), N, assoc)
    return out


def resampler_32f_xn(code, rem, step, shifts, N, assoc=1):
    code = _c(code, np.float32)
    shifts = _c(shifts, np.float32)
    out = np.empty((len(shifts), N), np.float32)
    lib().orc_resampler_32f_xn(_ptr(out), _ptr(code), rem, step, _ptr(shifts), len(code), len(shifts), N, assoc)
    return out


def high_dyn_resampler_32f_xn(code, rem, step, rate, shifts, N):
    code = _c(code, np.float32)
    shifts = _c(shifts, np.float32)
    out = np.empty((len(shifts), N), np.float32)
    lib().orc_high_dyn_resampler_32f_xn(_ptr(out), _ptr(code), rem, step, rate, _ptr(shifts), len(code),
                                        len(shifts), N)
    return out


def rotator_dot_prod_32fc_32f_xn(x, inc, phase, a):
    x = _c(x, np.complex64)
    a = _c(a, np.float32)
    K, N = a.shape
    ph = np.array([phase.real, phase.imag], np.float32)
    out = np.empty(K, np.complex64)
    lib().orc_rotator_dot_prod_32fc_32f_xn(_ptr(out), _ptr(x), float(inc.real), float(inc.imag), _ptr(ph),
                                           _ptr(a), K, N)
    return out, complex(ph[0], ph[1])


def rotator_dot_prod_32fc_32f_xn_avx(x, inc, phase, a):
    """The u_avx / a_avx rotator the reference dispatches on x86 (volk_oracle.c)."""
    x = _c(x, np.complex64)
    a = _c(a, np.float32)
    K, N = a.shape
    ph = np.array([phase.real, phase.imag], np.float32)
    out = np.empty(K, np.complex64)
    lib().orc_rotator_dot_prod_32fc_32f_xn_avx(_ptr(out), _ptr(x), float(inc.real), float(inc.imag), _ptr(ph),
                                               _ptr(a), K, N)
    return out, complex(ph[0], ph[1])


def s32f_sincos_32fc(phase_inc, N, phase=0.0):
    out = np.empty(N, np.complex64)
    ph = np.array([phase], np.float32)
    lib().orc_s32f_sincos_32fc(_ptr(out), phase_inc, _ptr(ph), N)
    return out


def s32f_sincos_32fc_avx2(phase_inc, N, phase=0.0):
    """The a_avx2 / u_avx2 protokernel (KERN/s32f_sincos_32fc.h:448-627)."""
    out = np.empty(N, np.complex64)
    ph = np.array([phase], np.float32)
    lib().orc_s32f_sincos_32fc_avx2(_ptr(out), phase_inc, _ptr(ph), N)
    return out


def index_max_32u(x):
    x = _c(x, np.float32)
    return int(lib().orc_index_max_32u(_ptr(x), len(x)))


def multicorrelator_real_codes(sig, code, shifts, rem_carr, carr_step, rem_code, code_step, N,
                               carr_rate=0.0, code_rate=0.0, high_dyn=False, assoc=1):
    """Cpu_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler (7-arg form)."""
    sig = _c(sig, np.complex64)
    code = _c(code, np.float32)
    shifts = _c(shifts, np.float32)
    out = np.empty(len(shifts), np.complex64)
    lib().orc_multicorrelator_real_codes(_ptr(out), _ptr(sig), _ptr(code), len(code), _ptr(shifts), len(shifts),
                                         rem_carr, carr_step, carr_rate, rem_code, code_step, code_rate, N,
                                         int(high_dyn), assoc)
    return out


def multicorrelator_real_codes_avx(sig, code, shifts, rem_carr, carr_step, rem_code, code_step, N):
    """The same call with the AVX rotator (u_avx / a_avx) the reference runs on x86."""
    sig = _c(sig, np.complex64)
    code = _c(code, np.float32)
    shifts = _c(shifts, np.float32)
    out = np.empty(len(shifts), np.complex64)
    lib().orc_multicorrelator_real_codes_avx(_ptr(out), _ptr(sig), _ptr(code), len(code), _ptr(shifts),
                                             len(shifts), rem_carr, carr_step, rem_code, code_step, N)
    return out


def multicorrelator_complex_codes(sig, code, shifts, rem_carr, carr_step, rem_code, code_step, N, assoc=1):
    """Cpu_Multicorrelator::Carrier_wipeoff_multicorrelator_resampler."""
    sig = _c(sig, np.complex64)
    code = _c(code, np.complex64)
    shifts = _c(shifts, np.float32)
    out = np.empty(len(shifts), np.complex64)
    lib().orc_multicorrelator_complex_codes(_ptr(out), _ptr(sig), _ptr(code), len(code), _ptr(shifts),
                                            len(shifts), rem_carr, carr_step, rem_code, code_step, N, assoc)
    return out


def multicorrelator_real_codes_exact(sig, code, shifts, rem_carr, carr_step, rem_code, code_step, N, assoc=1):
    sig = _c(sig, np.complex64)
    code = _c(code, np.float32)
    shifts = _c(shifts, np.float32)
    out = np.empty(2 * len(shifts), np.float64)
    lib().orc_multicorrelator_real_codes_exact(_ptr(out), _ptr(sig), _ptr(code), len(code), _ptr(shifts),
                                               len(shifts), rem_carr, carr_step, rem_code, code_step, N, assoc)
    return out[0::2] + 1j * out[1::2]
