"""CNF containers: the flat CSR literal/offset layout the kernels read from HBM.

A batch of formulas is three int32 arrays (see include/satmi.h):
    inst_clause_begin[B+1]  clause range of each instance
    clause_lit_begin[C+1]   literal range of each clause
    lits[L]                 DIMACS literals (the ints of REF.py's Clause = List[int])
plus inst_nvars[B] (largest variable index per instance).
"""
from dataclasses import dataclass

import numpy as np


@dataclass
class CnfBatch:
    inst_clause_begin: np.ndarray
    clause_lit_begin: np.ndarray
    lits: np.ndarray
    inst_nvars: np.ndarray

    @property
    def num_instances(self):
        return int(self.inst_nvars.shape[0])

    def maxima(self):
        """(max_vars, max_clauses, max_lits) over the batch."""
        icb = self.inst_clause_begin.astype(np.int64)
        clb = self.clause_lit_begin.astype(np.int64)
        ncl = np.diff(icb)
        nl = clb[icb[1:]] - clb[icb[:-1]]
        return (int(self.inst_nvars.max(initial=0)), int(ncl.max(initial=0)), int(nl.max(initial=0)))

    def instance(self, b):
        """Instance b back as List[List[int]]."""
        c0, c1 = int(self.inst_clause_begin[b]), int(self.inst_clause_begin[b + 1])
        out = []
        for c in range(c0, c1):
            out.append(self.lits[self.clause_lit_begin[c]:self.clause_lit_begin[c + 1]].tolist())
        return out


def pack(formulas):
    """Formulas (an iterable of iterables of clauses of int literals) -> CnfBatch.
    Literals must be nonzero and within int32 (INT32_MIN excluded: its negation
    does not exist); one-shot iterables are materialised once."""
    from itertools import chain
    formulas = [f if isinstance(f, (list, tuple)) else list(f) for f in formulas]
    formulas = [[c if isinstance(c, (list, tuple)) else list(c) for c in f] for f in formulas]
    ncl = np.fromiter((len(f) for f in formulas), dtype=np.int64, count=len(formulas))
    clen = np.fromiter((len(c) for f in formulas for c in f), dtype=np.int64, count=int(ncl.sum()))
    lits = np.fromiter(chain.from_iterable(chain.from_iterable(formulas)), dtype=np.int64, count=int(clen.sum()))
    if lits.size and not lits.all():
        raise ValueError("literal 0 is not allowed (REF.py:51)")
    if lits.size and (lits.max() > 2 ** 31 - 1 or lits.min() < -(2 ** 31 - 1)):
        raise ValueError("literals must lie within +-(2^31 - 1) (int32, the library's literal type)")
    icb = np.concatenate([[0], np.cumsum(ncl)])
    clb = np.concatenate([[0], np.cumsum(clen)])
    # largest variable per formula: the max |literal| over its literal range
    nv = np.zeros(len(formulas), dtype=np.int64)
    if lits.size:
        a = np.abs(lits)
        lo, hi = clb[icb[:-1]], clb[icb[1:]]
        has = hi > lo
        nv[has] = np.maximum.reduceat(a, lo[has])
    return CnfBatch(icb.astype(np.int32), clb.astype(np.int32),
                    (lits if lits.size else np.zeros(1, np.int64)).astype(np.int32), nv.astype(np.int32))


def uniform_ksat(num_instances, n, m, k, seed=0, dtype=np.int32):
    """Uniform random k-SAT: every clause has k distinct variables, each negated
    with probability 1/2 (the standard model behind 'random 3-SAT n=100,
    alpha=4.26').  Vectorised; returns a CnfBatch with fixed-size clauses."""
    rng = np.random.default_rng(seed)
    B = num_instances
    # k distinct variables per clause: sample with rejection of duplicates
    vars_ = rng.integers(1, n + 1, size=(B, m, k), dtype=np.int64)
    for _ in range(64):
        srt = np.sort(vars_, axis=2)
        dup = (np.diff(srt, axis=2) == 0).any(axis=2)
        if not dup.any():
            break
        vars_[dup] = rng.integers(1, n + 1, size=(int(dup.sum()), k), dtype=np.int64)
    else:
        raise RuntimeError("could not draw distinct variables")
    sign = rng.random(size=(B, m, k)) < 0.5
    lits = np.where(sign, -vars_, vars_).astype(dtype).reshape(-1)
    icb = (np.arange(B + 1, dtype=np.int64) * m).astype(np.int32)
    clb = (np.arange(B * m + 1, dtype=np.int64) * k)
    if clb[-1] >= 2 ** 31:
        raise ValueError("batch too large for int32 offsets; split it")
    return CnfBatch(icb, clb.astype(np.int32), lits.astype(np.int32), np.full(B, n, dtype=np.int32))


def menu_batch(count, num_clauses, max_literals_per_clause, num_variables, seed=0):
    """`count` formulas of generate_large_formula's distribution (REF.py:21-29:
    clause size uniform in 1..max, distinct variables, each negated w.p. 1/2),
    drawn with numpy for large batches (not the reference's draw sequence: use
    solvers.generate_large_formula under a seeded `random` for that)."""
    rng = np.random.default_rng(seed)
    C, k, n = count * num_clauses, max_literals_per_clause, num_variables
    if k > n:
        raise ValueError("more literals per clause than variables")
    size = rng.integers(1, k + 1, size=C)
    vars_ = np.argsort(rng.random((C, n)), axis=1)[:, :k] + 1       # a random k-subset, in random order
    lit = np.where(rng.random((C, k)) < 0.5, -vars_, vars_)
    lits = lit[np.arange(k)[None, :] < size[:, None]]
    clb = np.concatenate([[0], np.cumsum(size)])
    icb = np.arange(count + 1, dtype=np.int64) * num_clauses
    a = np.abs(lits)
    nv = np.maximum.reduceat(a, clb[icb[:-1]]) if count and num_clauses else np.zeros(count, np.int64)
    return CnfBatch(icb.astype(np.int32), clb.astype(np.int32), lits.astype(np.int32), nv.astype(np.int32))


def concat(batches):
    icb = [np.zeros(1, np.int64)]
    clb = [np.zeros(1, np.int64)]
    lits, nv = [], []
    c_off = 0
    l_off = 0
    for b in batches:
        icb.append(b.inst_clause_begin[1:].astype(np.int64) + c_off)
        clb.append(b.clause_lit_begin[1:].astype(np.int64) + l_off)
        nc = int(b.inst_clause_begin[-1])
        nl = int(b.clause_lit_begin[nc])
        lits.append(b.lits[:nl])
        nv.append(b.inst_nvars)
        c_off += nc
        l_off += nl
    return CnfBatch(np.concatenate(icb).astype(np.int32), np.concatenate(clb).astype(np.int32),
                    np.concatenate(lits + [np.zeros(1, np.int32)]).astype(np.int32)[:max(l_off, 1)],
                    np.concatenate(nv).astype(np.int32))


def pigeonhole(holes):
    """PHP(holes+1, holes) -- unsatisfiable; config [3] of BASELINE.json."""
    pig = holes + 1

    def x(p, h):
        return p * holes + h + 1

    cls = [[x(p, h) for h in range(holes)] for p in range(pig)]
    for h in range(holes):
        for p in range(pig):
            for q in range(p + 1, pig):
                cls.append([-x(p, h), -x(q, h)])
    return cls


def to_dimacs(formula, nvars=None):
    nv = nvars if nvars is not None else max([abs(l) for c in formula for l in c] + [0])
    lines = [f"p cnf {nv} {len(formula)}"]
    lines += [" ".join(str(l) for l in c) + " 0" for c in formula]
    return "\n".join(lines) + "\n"


def from_dimacs(text):
    """Parse DIMACS CNF (SATLIB uf/uuf files): 'c' comments, 'p cnf', '%' end marker."""
    formula, cur = [], []
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line[0] in "cp":
            continue
        if line[0] == "%":
            break
        for tok in line.split():
            v = int(tok)
            if v == 0:
                formula.append(cur)
                cur = []
            else:
                cur.append(v)
    if cur:
        formula.append(cur)
    return formula


def uniform_ksat_device(num_instances, n, m, k, seed, device):
    """uniform_ksat generated directly in HBM with torch (synthetic bench input).
    Returns (inst_clause_begin, clause_lit_begin, lits, inst_nvars) int32 tensors."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    B = num_instances
    vars_ = torch.randint(1, n + 1, (B, m, k), device=device, generator=g, dtype=torch.int32)
    for _ in range(64):
        srt, _ = torch.sort(vars_, dim=2)
        dup = (srt[:, :, 1:] == srt[:, :, :-1]).any(dim=2)
        nd = int(dup.sum())
        if nd == 0:
            break
        vars_[dup] = torch.randint(1, n + 1, (nd, k), device=device, generator=g, dtype=torch.int32)
    else:
        raise RuntimeError("could not draw distinct variables")   # as uniform_ksat
    sign = torch.rand((B, m, k), device=device, generator=g) < 0.5
    lits = torch.where(sign, -vars_, vars_).reshape(-1).contiguous()
    icb = (torch.arange(B + 1, device=device, dtype=torch.int64) * m).to(torch.int32)
    clb = (torch.arange(B * m + 1, device=device, dtype=torch.int64) * k).to(torch.int32)
    nv = torch.full((B,), n, device=device, dtype=torch.int32)
    return icb, clb, lits, nv
