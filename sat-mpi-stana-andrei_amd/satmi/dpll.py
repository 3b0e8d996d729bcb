"""Batched DPLL on the GPU (libsatmi.so, csrc/dpll.hip), host-array front end.

`dpll_batch` solves many formulas at once, one per wavefront.  Two semantics:

* mode="ref"   -- dpll_optimized exactly as REF.py:133-214: every solution
                  (leaf) in the reference's order, assignment dicts in the
                  reference's insertion order, counters equal to the reference's.
* mode="sound" -- the same procedure with each branch assignment applied to the
                  formula as a unit clause (propagated by REF.py's own
                  unit_propagate rule).  This is the complete DPLL decision
                  procedure the benchmark measures: SAT/UNSAT verdicts and models.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _capi
from .cnf import CnfBatch, pack


@dataclass
class DpllResult:
    status: np.ndarray      # [B] int32, _capi.DPLL_*
    counters: np.ndarray    # [B, 8] int64, _capi.COUNTER_NAMES
    sol_len: np.ndarray     # [B, sol_cap]
    sol_lits: np.ndarray    # [B, sol_cap, stride]
    root_len: np.ndarray    # [B]
    root_lits: np.ndarray   # [B, stride]

    def num_solutions(self, b):
        return int(self.counters[b, 5])

    def solutions(self, b):
        """Stored solutions of instance b as lists of signed literals (dict order)."""
        k = min(self.num_solutions(b), self.sol_len.shape[1])
        return [self.sol_lits[b, s, :self.sol_len[b, s]].tolist() for s in range(k)]

    def root_assignment(self, b):
        return self.root_lits[b, :self.root_len[b]].tolist()

    def counter_dict(self, b):
        return {n: int(self.counters[b, i]) for i, n in enumerate(_capi.COUNTER_NAMES[:7])}


def _ptr(a, t=ctypes.c_int32):
    return a.ctypes.data_as(ctypes.POINTER(t))


def dpll_batch(batch, mode="sound", max_solutions=1, node_limit=0, time_limit=0.0, sol_cap=None,
               inits=None):
    """Run batched DPLL.  `batch` is a CnfBatch or a list of formulas; `inits`
    an optional list (one per instance) of signed-literal lists (the caller's
    `assignment` dict of REF.py:133, in insertion order)."""
    if not isinstance(batch, CnfBatch):
        batch = pack(batch)
    L = _capi.load()
    _capi.require_gpu()
    B = batch.num_instances
    if sol_cap is None:
        sol_cap = max(1, max_solutions) if max_solutions > 0 else 1024
    nvars = int(batch.inst_nvars.max(initial=0))
    init_begin = init_lits = None
    if inits is not None:
        if len(inits) != B:
            raise ValueError("inits must have one entry per instance")
        init_begin = np.zeros(B + 1, dtype=np.int32)
        flat = []
        for b, a in enumerate(inits):
            flat.extend(int(x) for x in a)
            init_begin[b + 1] = len(flat)
            nvars = max([nvars] + [abs(int(x)) for x in a])
        init_lits = np.asarray(flat if flat else [0], dtype=np.int32)
    stride = max(1, nvars)
    status = np.zeros(B, dtype=np.int32)
    counters = np.zeros((B, _capi.NCOUNTERS), dtype=np.int64)
    sol_len = np.zeros((B, max(sol_cap, 1)), dtype=np.int32)
    sol_lits = np.zeros((B, max(sol_cap, 1), stride), dtype=np.int32)
    root_len = np.zeros(B, dtype=np.int32)
    root_lits = np.zeros((B, stride), dtype=np.int32)
    m = {"ref": _capi.MODE_REF, "sound": _capi.MODE_SOUND}[mode]
    rc = L.satmi_dpll_batch_host(
        B, _ptr(batch.inst_clause_begin), _ptr(batch.clause_lit_begin), _ptr(batch.lits),
        _ptr(batch.inst_nvars), _ptr(init_begin) if init_begin is not None else None,
        _ptr(init_lits) if init_lits is not None else None, m, int(max_solutions), int(node_limit),
        float(time_limit), int(sol_cap), int(stride), _ptr(status), _ptr(counters, ctypes.c_int64),
        _ptr(sol_len), _ptr(sol_lits), _ptr(root_len), _ptr(root_lits))
    _capi.check(rc, "satmi_dpll_batch_host")
    return DpllResult(status, counters, sol_len, sol_lits, root_len, root_lits)
