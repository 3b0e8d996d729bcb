"""CPU checks of the C ABI: the in-tree library loads and exports every symbol
include/satmi.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

from satmi import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "satmi.h")).read()
    return sorted(set(re.findall(r"\b(satmi_[a-z0-9_]+)\s*\(", text)))


def test_header_and_binding_agree():
    assert sorted(_capi.EXPORTED) == declared_symbols()


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libsatmi.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_capi.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name
    lib.satmi_abi_version.restype = ctypes.c_int
    assert lib.satmi_abi_version() == 1


def test_lds_layout_query():
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libsatmi.so not built")
    L = _capi.load()
    b100 = L.satmi_dpll_lds_bytes(100, 426, 1278)
    assert 0 < b100 < 16 * 1024
    assert L.satmi_dpll_lds_bytes(40000, 10, 10) == 0      # var codes are 15-bit
    assert L.satmi_dpll_lds_bytes(100, 100000, 100) == 0   # clause offsets are 16-bit
