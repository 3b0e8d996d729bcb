"""CDCL on the GPU (libsatmi.so, csrc/cdcl.hip): the reference's CDCLSolver /
cdcl_solve (REF.py:217-384), batched, one wavefront per formula.

`cdcl_batch(formulas, ...)` returns per formula the status, the assignment dict
(in insertion order) and the solver statistics; `cdcl_solve` is the
reference's entry point: (True, model) / (False, None).
"""
import ctypes

import numpy as np

from . import _capi
from .cnf import pack

CDCL_UNSAT, CDCL_SAT, CDCL_LIMIT, CDCL_ERROR, CDCL_FULL = 0, 1, -1, -2, -3
NSTATS = 8
STAT_NAMES = ("iterations", "conflicts", "decisions", "learned", "clauses", "watch_keys", "level", "pool_slots")


class CdclLimit(Exception):
    """The iteration / time bound or the arena stopped the solve loop (the
    reference's own loop has no bound: its caller times it out, REF.py:417-437)."""


def cdcl_batch(formulas, max_iter=0, time_limit=0.0, learn_cap=0):
    """Run cdcl_solve on every formula.  Returns a list of dicts: status
    (CDCL_*), assignment (signed literals, dict order), stats, var_inc."""
    return cdcl_batch_packed(pack(formulas), max_iter=max_iter, time_limit=time_limit, learn_cap=learn_cap)


def cdcl_batch_packed(batch, max_iter=0, time_limit=0.0, learn_cap=0, arrays=False):
    """cdcl_batch on a CnfBatch (the CSR host arrays of include/satmi.h).
    arrays=True returns the output arrays of satmi_cdcl_batch_host as they are
    (status[B], assign_len[B], assign[B, nv], stats[B, NSTATS], var_inc[B])
    instead of one dict per formula.  Calls from several host threads run
    concurrently on the device (each call has its own stream and arena)."""
    L = _capi.load()
    _capi.require_gpu()
    B = batch.num_instances
    nv = max([int(batch.inst_nvars.max()) if B else 0, 1])
    status = np.zeros(B, dtype=np.int32)
    alen = np.zeros(B, dtype=np.int32)
    assign = np.zeros((B, nv), dtype=np.int32)
    stats = np.zeros((B, NSTATS), dtype=np.int64)
    vinc = np.zeros(B, dtype=np.float64)
    P = ctypes.POINTER
    i32 = lambda a: a.ctypes.data_as(P(ctypes.c_int32))   # noqa: E731
    rc = L.satmi_cdcl_batch_host(B, i32(batch.inst_clause_begin), i32(batch.clause_lit_begin), i32(batch.lits),
                                 int(max_iter), int(learn_cap), float(time_limit), i32(status), i32(alen), i32(assign),
                                 nv, stats.ctypes.data_as(P(ctypes.c_int64)), vinc.ctypes.data_as(P(ctypes.c_double)))
    _capi.check(rc, "satmi_cdcl_batch_host")
    if arrays:
        return {"status": status, "assign_len": alen, "assign": assign, "stats": stats, "var_inc": vinc}
    return [{"status": int(status[b]), "assignment": assign[b, :alen[b]].tolist(),
             "stats": dict(zip(STAT_NAMES, stats[b].tolist())), "var_inc": float(vinc[b])} for b in range(B)]


def cdcl_solve(formula, time_limit=0.0, learn_cap=1 << 24):
    """cdcl_solve(formula) -> (bool, Optional[dict]) (REF.py:382-384).  Like the
    reference, `formula` is the list the solver appends its learned clauses to
    (REF.py:349-350) -- here it is left as given (the GPU keeps its own copy).
    Raises CdclLimit where the reference would still be running at the deadline,
    and KeyError where the reference raises one (REF.py:312, :342)."""
    r = cdcl_batch([formula], time_limit=time_limit, learn_cap=learn_cap)[0]
    if r["status"] == CDCL_SAT:
        return True, {abs(l): l > 0 for l in r["assignment"]}
    if r["status"] == CDCL_UNSAT:
        return False, None
    if r["status"] == CDCL_ERROR:
        raise KeyError("analyze_conflict reached an unassigned variable (the reference raises KeyError here)")
    raise CdclLimit(f"CDCL stopped after {r['stats']['iterations']} iterations "
                    f"({'arena full' if r['status'] == CDCL_FULL else 'time or iteration limit'})")


def last_stats():
    """The calling thread's last CDCL launch: span (s, device wall clock), busy
    wave-time (s) and resident waves; utilisation = busy / (resident x span)."""
    import ctypes
    L = _capi.load()
    span, busy, res = ctypes.c_double(0.0), ctypes.c_double(0.0), ctypes.c_int(0)
    _capi.check(L.satmi_cdcl_last_stats(ctypes.byref(span), ctypes.byref(busy), ctypes.byref(res)),
                "satmi_cdcl_last_stats")
    util = busy.value / (res.value * span.value) if res.value and span.value > 0 else None
    return {"span_s": span.value, "busy_wave_s": busy.value, "resident_waves": res.value, "wave_utilisation": util}
