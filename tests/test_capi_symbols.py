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
    assert lib.satmi_abi_version() == 2


def test_lds_layout_query():
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libsatmi.so not built")
    L = _capi.load()
    b100 = L.satmi_dpll_lds_bytes(100, 426, 1278)
    assert 0 < b100 < 16 * 1024
    assert L.satmi_dpll_lds_bytes(40000, 10, 10) == 0      # var codes are 15-bit
    assert L.satmi_dpll_lds_bytes(100, 100000, 100) == 0   # clause offsets are 16-bit


def test_scan_kernel_eligibility_query():
    """The clause-scan kernel's LDS image and eligibility (host-side layout only)."""
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libsatmi.so not built")
    L = _capi.load()
    s100 = L.satmi_dpll_scan_lds_bytes(100, 426, 1278, 3)
    assert 0 < s100 <= 6 * 1024 < L.satmi_dpll_lds_bytes(100, 426, 1278)
    assert L.satmi_dpll_scan_lds_bytes(200, 4223, 21115, 5) > 0          # configs[4] 5-SAT
    assert L.satmi_dpll_scan_lds_bytes(600, 100, 300, 3) > 0             # > 511 vars: 12-bit codes
    assert L.satmi_dpll_scan_lds_bytes(100, 426, 1278, 6) == 0           # clauses of <= 5 literals
    assert L.satmi_dpll_scan_lds_bytes(100, 426, 1278, 0) == 0           # unknown / empty clause
    assert L.satmi_dpll_scan_lds_bytes(3000, 426, 1278, 3) == 0          # <= 2047 variables
    # the plan follows the policy: REF mode and caller assignments use the general kernel
    assert _capi.plan(100, 426, 1278, 3, _capi.MODE_REF)[0] == _capi.KERNEL_GENERAL
    assert _capi.plan(100, 426, 1278, 3, _capi.MODE_SOUND, has_init=True)[0] == _capi.KERNEL_GENERAL
    kern, lds_inc, _ = _capi.plan(100, 426, 1278, 3)
    assert kern == _capi.KERNEL_INC    # SOUND mode default: incremental rounds
    _capi.set_kernel(_capi.KERNEL_SCAN)
    try:
        kern, lds, _ = _capi.plan(100, 426, 1278, 3)
    finally:
        _capi.set_kernel(_capi.KERNEL_AUTO)
    # the launch's real per-wave LDS: one-wave workgroups keep the literal states
    # in a 256-B static array instead of the image's 2(n+1) = 202 B (+ alignment),
    # (n <= 127) byte-wide trail / frames / snapshot: 3 x (208 - 112) + (512 - 432)
    # (16-bit codes keep 256 snapshot entries in LDS, byte codes all 427), and one
    # counter word per literal code (816 B) where the 16-bit-code layout of
    # satmi_dpll_scan_lds_bytes packs two per word (416 B)
    assert kern == _capi.KERNEL_SCAN and s100 - 208 + 256 - 3 * 96 - (512 - 432) + (816 - 416) == lds
    # the bench class (K=3, n <= 127, m <= 448) runs the static-layout incremental
    # kernel: 5,108 B per wave whatever the instance size, 32 waves per CU
    assert lds_inc == 5108 and _capi.plan(50, 213, 639, 3)[1] == 5108
    # beyond it, the runtime layout: + occurrence-list offsets (2(2n+3) B) and the
    # unit bitmap with its prefixes (8 B per 32 clauses)
    kern, lds_big, _ = _capi.plan(130, 426, 1278, 3)
    _capi.set_kernel(_capi.KERNEL_SCAN)
    try:
        lds_big_scan = _capi.plan(130, 426, 1278, 3)[1]
    finally:
        _capi.set_kernel(_capi.KERNEL_AUTO)
    # (the incremental plan may take multi-wave workgroups when they keep more
    # waves resident: the literal states then move from the 512-B static array
    # into each wave's image, 2(n+1) = 262 -> 272 B)
    assert kern == _capi.KERNEL_INC and lds_big in (lds_big_scan + 528 + 112, lds_big_scan - 512 + 272 + 528 + 112)
    _capi.set_kernel(_capi.KERNEL_GENERAL)
    try:
        assert _capi.plan(100, 426, 1278, 3)[0] == _capi.KERNEL_GENERAL
    finally:
        _capi.set_kernel(_capi.KERNEL_AUTO)
    with pytest.raises(_capi.SatmiError):
        _capi.set_kernel(7)


def test_split_policy_arguments():
    """satmi_dpll_set_split: 0 off / 1 auto / 2 always, helpers in [0, 32];
    satmi_dpll_set_split_warmup: < 0 restores the default (host-side state only)."""
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libsatmi.so not built")
    try:
        for mode in (_capi.SPLIT_OFF, _capi.SPLIT_ALWAYS, _capi.SPLIT_AUTO):
            _capi.set_split(mode)
        with pytest.raises(_capi.SatmiError):
            _capi.set_split(3)
        with pytest.raises(_capi.SatmiError):
            _capi.set_split(_capi.SPLIT_AUTO, helpers_per_cu=33)
        _capi.set_split_warmup(0)
        _capi.set_split_warmup(1000)
    finally:
        _capi.set_split(_capi.SPLIT_AUTO)
        _capi.set_split_warmup(-1)
