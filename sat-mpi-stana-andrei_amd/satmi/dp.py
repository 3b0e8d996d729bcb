"""Davis-Putnam elimination on the GPU (libsatmi.so, csrc/dp.hip).

`eliminate(formula, ...)` runs REF.py:98-130 step by step -- variables in the
reference's own order (CPython's `set.pop()`, modelled on the device) -- and can
return every intermediate clause list; `davis_putnam_solve` is the reference's
boolean entry point.
"""
import ctypes

import numpy as np

from . import _capi
from .resolution import _csr, _p


class DavisPutnamLimit(Exception):
    """A step / clause / time limit stopped the elimination before a verdict."""


def eliminate(formula, step_limit=0, clause_limit=0, time_limit=0.0, record=False, rec_cap=1 << 22):
    """Returns {"result": 1 (True) | 0 (False) | -1 (limit), "vars": [eliminated
    variable per step], "steps": int, "clauses": [clause list after each completed
    step, every clause in its Python set iteration order] (record=True)}."""
    L = _capi.load()
    _capi.require_gpu()
    off, lits = _csr(formula)
    nv = max(int(np.abs(lits.astype(np.int64)).max()) if len(formula) and off[-1] else 1, 1)
    res = ctypes.c_int32(0)
    steps = ctypes.c_int32(0)
    trace = np.zeros(nv + 1, dtype=np.int32)
    if record:
        rl = np.zeros(rec_cap, dtype=np.int32)
        rco = np.zeros(rec_cap + 1, dtype=np.int64)
        rso = np.full(nv + 2, -1, dtype=np.int64)   # untouched (-1) for a step that ended the search
        rc = L.satmi_dp_host(len(formula), _p(off), _p(lits), int(step_limit), int(clause_limit), float(time_limit),
                             ctypes.byref(res), _p(trace), nv + 1, ctypes.byref(steps), _p(rl), rec_cap,
                             _p(rco, ctypes.c_int64), rec_cap + 1, _p(rso, ctypes.c_int64), nv + 2)
    else:
        rc = L.satmi_dp_host(len(formula), _p(off), _p(lits), int(step_limit), int(clause_limit), float(time_limit),
                             ctypes.byref(res), _p(trace), nv + 1, ctypes.byref(steps), None, 0, None, 0, None, 0)
    _capi.check(rc, "satmi_dp_host")
    n = steps.value
    out = {"result": res.value, "vars": trace[:min(n, nv + 1)].tolist(), "steps": n}
    if record:
        done = []
        for s in range(min(n, nv + 1)):
            if rso[s + 1] < 0:
                break
            done.append([rl[rco[c]:rco[c + 1]].tolist() for c in range(rso[s], rso[s + 1])])
        out["clauses"] = done
    return out


def last_stats():
    """Work of the last eliminate() call in this thread (satmi_dp_last_stats):
    steps, subset tests, new resolvents, kernel launches, key words and the
    device time of the elimination steps (ms)."""
    v = [ctypes.c_int64(0) for _ in range(4)]
    w = ctypes.c_int(0)
    ms = ctypes.c_double(0.0)
    _capi.check(_capi.load().satmi_dp_last_stats(*(ctypes.byref(x) for x in v), ctypes.byref(w), ctypes.byref(ms)),
                "satmi_dp_last_stats")
    return {"steps": v[0].value, "subset_tests": v[1].value, "new_clauses": v[2].value,
            "launches": v[3].value, "words": w.value, "device_ms": ms.value}


def davis_putnam_solve(formula, time_limit=0.0):
    """davis_putnam_solver(formula) -> bool (REF.py:98-130)."""
    r = eliminate(formula, time_limit=time_limit)
    if r["result"] < 0:
        raise DavisPutnamLimit(f"Davis-Putnam stopped by its limit after {r['steps']} steps")
    return bool(r["result"])
