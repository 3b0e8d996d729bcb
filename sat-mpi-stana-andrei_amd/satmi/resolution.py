"""Resolution saturation on the GPU (libsatmi.so, csrc/resolution.hip).

`resolve(formula, ...)` runs REF.py:63-95's saturation and returns the verdict
plus, optionally, the set of clauses each pass added; `resolution_solve` is the
reference's boolean entry point.
"""
import ctypes
import itertools

import numpy as np

from . import _capi


class ResolutionLimit(Exception):
    """A pass / clause / time limit stopped the saturation before a verdict."""


def _csr(formula):
    """The formula's CSR host arrays (clause offsets, literals), built without a
    per-literal Python loop (a call's conversion is part of its time)."""
    off = np.zeros(len(formula) + 1, dtype=np.int32)
    np.cumsum(np.fromiter(map(len, formula), dtype=np.int32, count=len(formula)), out=off[1:])
    n = int(off[-1])
    if n == 0:
        return off, np.zeros(1, dtype=np.int32)
    # (a literal outside int32 raises OverflowError here, like np.asarray did)
    flat = np.fromiter(itertools.chain.from_iterable(formula), dtype=np.int32, count=n)
    if not flat.all():
        raise ValueError("literal 0 is not allowed (REF.py:51)")
    return off, flat


def _p(a, t=ctypes.c_int32):
    return a.ctypes.data_as(ctypes.POINTER(t))


def resolve(formula, max_passes=0, clause_limit=0, time_limit=0.0, record=False, rec_cap=1 << 22):
    """Returns {"result": 1 (True) | 0 (False) | -1 (limit), "passes": int,
    "pass_new": [...], "clauses": [[sorted clause, ...] per pass] (record=True)}."""
    L = _capi.load()
    _capi.require_gpu()
    off, lits = _csr(formula)
    res = ctypes.c_int32(0)
    passes = ctypes.c_int32(0)
    pcap = int(max_passes) if 0 < max_passes < (1 << 16) else 1 << 16
    pass_new = np.zeros(pcap, dtype=np.int64)
    if record:
        rl = np.zeros(rec_cap, dtype=np.int32)
        rco = np.zeros(rec_cap + 1, dtype=np.int64)
        rpo = np.zeros(pcap + 1, dtype=np.int64)
        rc = L.satmi_resolution_host(len(formula), _p(off), _p(lits), int(max_passes), int(clause_limit),
                                     float(time_limit), ctypes.byref(res), ctypes.byref(passes),
                                     _p(pass_new, ctypes.c_int64), pcap, _p(rl), rec_cap,
                                     _p(rco, ctypes.c_int64), rec_cap + 1, _p(rpo, ctypes.c_int64), pcap + 1)
    else:
        rc = L.satmi_resolution_host(len(formula), _p(off), _p(lits), int(max_passes), int(clause_limit),
                                     float(time_limit), ctypes.byref(res), ctypes.byref(passes),
                                     _p(pass_new, ctypes.c_int64), pcap, None, 0, None, 0, None, 0)
    _capi.check(rc, "satmi_resolution_host")
    n = passes.value
    out = {"result": res.value, "passes": n, "pass_new": pass_new[:min(n, pcap)].tolist()}
    if record:
        out["clauses"] = [[rl[rco[c]:rco[c + 1]].tolist() for c in range(rpo[p], rpo[p + 1])]
                          for p in range(min(n, pcap))]
    return out


def last_stats():
    """Work and device time of the last resolve() call: pairs, candidate
    resolvents, pair-kernel ms, claim (hash dedup) kernel ms, and the pass
    kernels' live shader clock (Hz; 0 on the general path)."""
    L = _capi.load()
    pairs, cand = ctypes.c_int64(0), ctypes.c_int64(0)
    pms, cms = ctypes.c_double(0.0), ctypes.c_double(0.0)
    _capi.check(L.satmi_resolution_last_stats(ctypes.byref(pairs), ctypes.byref(cand), ctypes.byref(pms),
                                              ctypes.byref(cms)), "satmi_resolution_last_stats")
    hz = ctypes.c_double(0.0)
    _capi.check(L.satmi_resolution_last_clock(ctypes.byref(hz)), "satmi_resolution_last_clock")
    return {"pairs": pairs.value, "candidates": cand.value, "pair_ms": pms.value, "claim_ms": cms.value,
            "shader_clock_hz": hz.value}


def resolution_solve(formula, time_limit=0.0):
    """resolution_solver(formula) -> bool (REF.py:63-95)."""
    r = resolve(formula, time_limit=time_limit)
    if r["result"] < 0:
        raise ResolutionLimit(f"resolution stopped by its limit after {r['passes']} passes")
    return bool(r["result"])
