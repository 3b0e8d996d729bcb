"""ctypes front-end for the CPU oracle (liboracle.so built from oracle/*.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, by __graft_entry__.smoke() as the
checker and by bench.py's cpu_baseline leg.  The product package never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in
                ("nodes", "decisions", "unit_props", "pure_assigns", "conflicts", "solutions")]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.POINTER
        i32p, i64p = P(ctypes.c_int32), P(ctypes.c_int64)
        L.oracle_dpll.restype = ctypes.c_int
        L.oracle_dpll.argtypes = [ctypes.c_int, ctypes.c_int, i32p, i32p, ctypes.c_int, ctypes.c_int64,
                                  ctypes.c_int64, i32p, ctypes.c_int, i32p, ctypes.c_int64, i64p,
                                  ctypes.c_int64, i32p, P(ctypes.c_int), P(Counters)]
        L.oracle_dp.restype = ctypes.c_int
        L.oracle_dp.argtypes = [ctypes.c_int, i32p, i32p, ctypes.c_int64, ctypes.c_int64, i32p, ctypes.c_int,
                                P(ctypes.c_int), i32p, ctypes.c_int64, i64p, ctypes.c_int64, i64p, ctypes.c_int]
        L.oracle_resolution.restype = ctypes.c_int
        L.oracle_resolution.argtypes = [ctypes.c_int, i32p, i32p, ctypes.c_int, ctypes.c_int64, i64p,
                                        ctypes.c_int, P(ctypes.c_int), i32p, ctypes.c_int64, i64p,
                                        ctypes.c_int64, i64p, ctypes.c_int]
        L.oracle_cdcl.restype = ctypes.c_int
        L.oracle_cdcl.argtypes = [ctypes.c_int, i32p, i32p, ctypes.c_int64, i32p, P(ctypes.c_int32), i64p,
                                  P(ctypes.c_double)]
        L.pyset_probe_from_list.restype = ctypes.c_int
        L.pyset_probe_from_list.argtypes = [i64p, ctypes.c_int, i64p]
        L.pyset_probe_resolvent.restype = ctypes.c_int
        L.pyset_probe_resolvent.argtypes = [i64p, ctypes.c_int, ctypes.c_int64, i64p, ctypes.c_int,
                                            ctypes.c_int64, i64p]
        L.pyset_probe_var_pop.restype = ctypes.c_int64
        L.pyset_probe_var_pop.argtypes = [i64p, P(ctypes.c_int), ctypes.c_int]
        _lib = L
    return _lib


def _csr(formula):
    off = np.zeros(len(formula) + 1, dtype=np.int32)
    for i, c in enumerate(formula):
        off[i + 1] = off[i] + len(c)
    lits = np.array([l for c in formula for l in c] or [0], dtype=np.int32)
    return off, lits


def _p(a, t=ctypes.c_int32):
    return a.ctypes.data_as(ctypes.POINTER(t))


def dpll(formula, mode="ref", max_solutions=0, node_limit=0, init=None, sol_cap=1 << 16):
    """Run the DPLL restatement.  mode 'ref' = REF.py:133-214 exactly; 'sound' =
    decisions applied as unit clauses.  Returns dict with status, solutions
    (lists of signed literals in assignment-dict order), counters, root_assign."""
    off, lits = _csr(formula)
    nv = max([abs(l) for c in formula for l in c] + [abs(l) for l in (init or [])] + [1])
    init_a = np.array(list(init or []) or [0], dtype=np.int32)
    cap_l = max(1, sol_cap * (nv + 1))
    sol_lits = np.zeros(cap_l, dtype=np.int32)
    sol_off = np.zeros(sol_cap + 1, dtype=np.int64)
    root = np.zeros(nv + 1, dtype=np.int32)
    root_len = ctypes.c_int(0)
    ctr = Counters()
    st = lib().oracle_dpll(nv, len(formula), _p(off), _p(lits), 0 if mode == "ref" else 1,
                           max_solutions, node_limit, _p(init_a), len(init or []),
                           _p(sol_lits), cap_l, _p(sol_off, ctypes.c_int64), sol_cap,
                           _p(root), ctypes.byref(root_len), ctypes.byref(ctr))
    nsol = min(ctr.solutions, sol_cap)
    sols = [sol_lits[sol_off[k]:sol_off[k + 1]].tolist() for k in range(nsol)]
    return {"status": st, "solutions": sols,
            "counters": {n: getattr(ctr, n) for n, _ in Counters._fields_},
            "root_assign": root[:root_len.value].tolist()}


def dp(formula, step_limit=0, clause_limit=0, record=False, rec_cap=1 << 20):
    off, lits = _csr(formula)
    nv = max([abs(l) for c in formula for l in c] + [1])
    trace = np.zeros(nv + 1, dtype=np.int32)
    nsteps = ctypes.c_int(0)
    if record:
        rl = np.zeros(rec_cap, dtype=np.int32)
        rco = np.zeros(rec_cap + 1, dtype=np.int64)
        rso = np.zeros(nv + 2, dtype=np.int64)
        r = lib().oracle_dp(len(formula), _p(off), _p(lits), step_limit, clause_limit, _p(trace), nv + 1,
                            ctypes.byref(nsteps), _p(rl), rec_cap, _p(rco, ctypes.c_int64), rec_cap,
                            _p(rso, ctypes.c_int64), nv + 1)
    else:
        r = lib().oracle_dp(len(formula), _p(off), _p(lits), step_limit, clause_limit, _p(trace), nv + 1,
                            ctypes.byref(nsteps), None, 0, None, 0, None, 0)
    out = {"result": r, "vars": trace[:min(nsteps.value, nv + 1)].tolist(), "steps": nsteps.value}
    if record:
        steps = []
        for s in range(min(nsteps.value, nv + 1)):
            if rso[s + 1] < rso[s]:
                break
            cl = [rl[rco[c]:rco[c + 1]].tolist() for c in range(rso[s], rso[s + 1])]
            steps.append(cl)
        out["clauses"] = steps
    return out


def resolution(formula, max_passes=0, clause_limit=0, record=False, rec_cap=1 << 20):
    off, lits = _csr(formula)
    pass_new = np.zeros(4096, dtype=np.int64)
    npass = ctypes.c_int(0)
    if record:
        rl = np.zeros(rec_cap, dtype=np.int32)
        rco = np.zeros(rec_cap + 1, dtype=np.int64)
        rpo = np.zeros(4097, dtype=np.int64)
        r = lib().oracle_resolution(len(formula), _p(off), _p(lits), max_passes, clause_limit,
                                    _p(pass_new, ctypes.c_int64), 4096, ctypes.byref(npass), _p(rl), rec_cap,
                                    _p(rco, ctypes.c_int64), rec_cap, _p(rpo, ctypes.c_int64), 4096)
    else:
        r = lib().oracle_resolution(len(formula), _p(off), _p(lits), max_passes, clause_limit,
                                    _p(pass_new, ctypes.c_int64), 4096, ctypes.byref(npass), None, 0, None, 0,
                                    None, 0)
    out = {"result": r, "passes": npass.value, "pass_new": pass_new[:npass.value].tolist()}
    if record:
        out["clauses"] = [[rl[rco[c]:rco[c + 1]].tolist() for c in range(rpo[p], rpo[p + 1])]
                          for p in range(npass.value)]
    return out


def pyset_from_list(keys):
    a = np.array(list(keys) or [0], dtype=np.int64)
    out = np.zeros(max(1, len(keys)), dtype=np.int64)
    n = lib().pyset_probe_from_list(_p(a, ctypes.c_int64), len(keys), _p(out, ctypes.c_int64))
    return out[:n].tolist()


def pyset_resolvent(a, x, b, y):
    A = np.array(list(a) or [0], dtype=np.int64)
    B = np.array(list(b) or [0], dtype=np.int64)
    out = np.zeros(len(a) + len(b) + 1, dtype=np.int64)
    n = lib().pyset_probe_resolvent(_p(A, ctypes.c_int64), len(a), x, _p(B, ctypes.c_int64), len(b), y,
                                    _p(out, ctypes.c_int64))
    return out[:n].tolist()


def pyset_var_pop(lists):
    off = np.zeros(len(lists) + 1, dtype=np.int32)
    for i, c in enumerate(lists):
        off[i + 1] = off[i] + len(c)
    lits = np.array([l for c in lists for l in c] or [0], dtype=np.int64)
    return lib().pyset_probe_var_pop(_p(lits, ctypes.c_int64), _p(off, ctypes.c_int), len(lists))


CDCL_STATS = ("iterations", "conflicts", "decisions", "learned", "clauses", "watch_keys", "level")


def cdcl(formula, max_iter=0):
    """cdcl_solve (REF.py:382-384) restated: {"result": 1 True | 0 False | -1 the
    iteration cap | -2 the reference raises, "assignment": the assignment dict as
    signed literals in insertion order (the model for result 1), "var_inc",
    "stats": CDCL_STATS}."""
    off, lits = _csr(formula)
    nv = max([abs(l) for c in formula for l in c] + [1])
    model = np.zeros(nv + 1, dtype=np.int32)
    mlen = ctypes.c_int32(0)
    st = np.zeros(len(CDCL_STATS), dtype=np.int64)
    vi = ctypes.c_double(0.0)
    r = lib().oracle_cdcl(len(formula), _p(off), _p(lits), int(max_iter), _p(model), ctypes.byref(mlen),
                          _p(st, ctypes.c_int64), ctypes.byref(vi))
    return {"result": r, "assignment": model[:mlen.value].tolist(), "var_inc": vi.value,
            "stats": dict(zip(CDCL_STATS, st.tolist()))}
