"""CPU-side checks of the C-ABI library: it builds, loads, and exports every entry point that
include/deltareplay.h declares (no compute calls: there is no GPU in the CPU suite)."""
import ctypes
import os
import re

from tests.conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "deltareplay.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dr_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_symbols():
    from delta_amd import _native as N
    assert _declared() == sorted(N.SYMBOLS)


def test_library_exports_every_declared_symbol():
    from delta_amd import _native as N
    lib = ctypes.CDLL(N.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name
    assert N.load().dr_abi_version() == N.ABI_VERSION == 4  # include/deltareplay.h DR_ABI_VERSION


def test_no_device_is_reported_loudly():
    """Without a GPU the product path must fail with DR_E_DEVICE, never fall back to the CPU."""
    import torch
    if torch.cuda.is_available():
        return
    from delta_amd import _native as N
    lib = N.load()
    ctx = ctypes.c_void_p()
    assert lib.dr_ctx_create(0, ctypes.byref(ctx)) == 14
