"""C-ABI boundary checks that need no GPU: the library loads, exports exactly what
include/gsdr.h declares, struct layouts agree, and calls fail cleanly (no crash)
when no device is present."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import gsdr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gsdr.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(gsdr_[a-z0-9_]+)\s*\(", txt)))


def test_header_declarations_match_binding_list():
    assert _declared() == sorted(gsdr.EXPORTED)


def test_library_exports_every_declared_symbol():
    L = gsdr.load()
    for name in _declared():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", gsdr.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (gsdr_[a-z0-9_]+)", out))
    assert exported == set(_declared())


def test_abi_version():
    assert gsdr.load().gsdr_abi_version() == 1


def test_struct_layouts_match_c_compiler(tmp_path):
    """ctypes mirrors vs the C compiler's sizeof/offsetof of the header structs."""
    src = tmp_path / "layout.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gsdr.h"', "int main(void){"]
    for cname, py in (("gsdr_acq_conf", gsdr.AcqConf), ("gsdr_acq_result", gsdr.AcqResult),
                      ("gsdr_corr_job", gsdr.CorrJob)):
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0;}")
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(l.split() for l in subprocess.check_output([str(exe)], text=True).splitlines())
    for cname, py in (("gsdr_acq_conf", gsdr.AcqConf), ("gsdr_acq_result", gsdr.AcqResult),
                      ("gsdr_corr_job", gsdr.CorrJob)):
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[cname + "." + f]) == getattr(py, f).offset, (cname, f)


def test_null_arguments_are_rejected():
    L = gsdr.load()
    assert L.gsdr_acq_create(0, None, None) == gsdr.GSDR_E_ARG
    assert b"null" in L.gsdr_last_error()
    assert L.gsdr_corr_create(0, 1, 1, 1, None) == gsdr.GSDR_E_ARG
    assert L.gsdr_acq_set_threshold(None, 1.0) == gsdr.GSDR_E_ARG


def test_create_without_device_fails_cleanly():
    if gsdr.device_count() > 0:
        pytest.skip("a GPU is present; covered by the gpu tests")
    with pytest.raises(gsdr.GsdrError):
        gsdr.Acquisition(4000000, 4000, 10000, 250)
    with pytest.raises(gsdr.GsdrError):
        gsdr.Correlator(4, 16000)


def test_tracking_struct_layouts_match_c_compiler(tmp_path):
    """numpy mirrors of gsdr_trk_conf / gsdr_trk_epoch vs sizeof/offsetof."""
    src = tmp_path / "trk_layout.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gsdr.h"', "int main(void){"]
    pairs = (("gsdr_trk_conf", gsdr.TRK_CONF_DTYPE), ("gsdr_trk_epoch", gsdr.TRK_EPOCH_DTYPE))
    for cname, dt in pairs:
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in dt.names:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0;}")
    src.write_text("\n".join(lines))
    exe = tmp_path / "trk_layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(l.split() for l in subprocess.check_output([str(exe)], text=True).splitlines())
    for cname, dt in pairs:
        assert int(got[cname]) == dt.itemsize, cname
        for f in dt.names:
            assert int(got[cname + "." + f]) == dt.fields[f][1], (cname, f)


def test_tracking_conf_default_is_host_only():
    """gsdr_trk_conf_default needs no device and carries Dll_Pll_Conf's defaults."""
    c = gsdr.trk_conf_default()
    assert float(c["fs_in"][0]) == 2000000.0
    assert int(c["cn0_samples"][0]) == 20 and int(c["cn0_min"][0]) == 25
    assert int(c["pll_filter_order"][0]) == 3 and int(c["dll_filter_order"][0]) == 2
    assert abs(float(c["carrier_lock_th"][0]) - 0.7) < 1e-12
    if gsdr.device_count() == 0:
        with pytest.raises(gsdr.GsdrError):
            gsdr.Tracking(c)
