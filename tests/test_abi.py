"""The C-ABI library loads and exports every symbol include/fitgpu.h declares (no compute calls)."""
import ctypes as C
import os
import re

import pytest

from fitgpu import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "fitgpu.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|int32_t|int64_t|const char\*)\s+\**(fit_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    assert declared() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared():
        assert hasattr(L, name), name


def test_abi_version_and_strerror():
    L = _lib.lib()
    assert L.fit_abi_version() == 8
    assert L.fit_strerror(_lib.FIT_E_NODEV) == b"no usable gfx950 device"


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure mode")
def test_no_cpu_fallback_fails_loudly():
    import fitgpu
    with pytest.raises(fitgpu.FitError) as ei:
        fitgpu.Engine()
    assert ei.value.code == _lib.FIT_E_NODEV


def test_null_args_are_rejected():
    L = _lib.lib()
    h = C.c_void_p()
    assert L.fit_create(None, None) == _lib.FIT_E_INVAL
    assert L.fit_load_nodes(None, 0, None, None, None, None, None) == _lib.FIT_E_INVAL
    assert L.fit_place(None, 0, None, None, None, None, None, None, 1, None, None) == _lib.FIT_E_INVAL
    del h
    a = C.c_void_p()
    assert L.fit_admitter_create(None, 16, 1000, C.byref(a)) == _lib.FIT_E_INVAL
    assert L.fit_admit(None, None, None) == _lib.FIT_E_INVAL
    assert L.fit_admitter_load_nodes(None, 0, None, None, None, None, None) == _lib.FIT_E_INVAL
    L.fit_admitter_destroy(None)  # no-op
