"""The C-ABI library loads and exports every symbol include/rmbx.h declares (CPU, no compute)."""

import ctypes
import os
import re

from conftest import ROOT

from robomanipbaselines_amd import _native as N


def _declared():
    txt = open(os.path.join(ROOT, "include", "rmbx.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rmbx_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    lib = N.load()
    names = _declared()
    assert len(names) >= 8
    for n in names:
        assert hasattr(lib, n), f"{n} declared in rmbx.h but not exported"
        assert n in N.SIGNATURES, f"{n} has no ctypes signature in _native.SIGNATURES"


def test_signatures_cover_only_declared():
    assert set(N.SIGNATURES) == set(_declared())


def test_abi_version_and_errors():
    lib = N.load()
    assert lib.rmbx_abi_version() == 2
    cnt = ctypes.c_int(-5)
    assert lib.rmbx_device_count(ctypes.byref(cnt)) == 0
    assert cnt.value >= 0
    # argument validation happens before any device call
    st = lib.rmbx_cable_reward(None, None, None, None, None, 4, 25, None)
    assert st == -1
    assert b"NULL" in lib.rmbx_last_error()
