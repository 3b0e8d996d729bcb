"""Drop-in solver entry points of the reference script, backed by the GPU.

Same names, signatures, argument meaning and return values as
REF.py ("comparatie intre algoritmii de rezolvare a seturilor de clauze.py"):

    generate_large_formula(num_clauses, max_literals_per_clause, num_variables)  REF.py:21-29
    resolution_solver(formula) -> bool                                           REF.py:63-95
    davis_putnam_solver(formula) -> bool                                         REF.py:98-130
    dpll_optimized(formula, assignment=None) -> List[Assignment]                 REF.py:133-214
    cdcl_solve(formula) -> Tuple[bool, Optional[Assignment]]                     REF.py:217-384
    hybrid_solver(formula, threshold=1000) -> List[Assignment]                   REF.py:400-404
    pysat_solver(formula) -> List[Assignment]                                    REF.py:387-397

The solvers run on the MI355X through libsatmi.so; there is no CPU fallback.
"""
import random
from typing import Dict, List, Optional, Tuple

from . import _capi
from .dpll import dpll_batch

Literal = int
Clause = List[Literal]
Formula = List[Clause]
Assignment = Dict[int, bool]

# Per-call wall-clock limit (seconds) the comparison driver sets around a solver
# call (REF.py:417-437 runs each solver under a 60 s timeout); 0 = unlimited.
_time_limit = 0.0


class SolverTimeout(Exception):
    pass


def set_time_limit(seconds):
    global _time_limit
    _time_limit = float(seconds or 0.0)


def generate_large_formula(num_clauses: int, max_literals_per_clause: int, num_variables: int) -> Formula:
    """Random CNF, drawing from Python's `random` in the same sequence as REF.py:21-29
    (size ~ randint(1, max), distinct variables by sample(), each negated w.p. 1/2),
    so a seeded `random` produces the reference's formula."""
    pool = range(1, num_variables + 1)
    out: Formula = []
    for _ in range(num_clauses):
        size = random.randint(1, max_literals_per_clause)
        chosen = random.sample(pool, size)
        out.append([v if random.random() < 0.5 else -v for v in chosen])
    return out


def dpll_optimized(formula: Formula, assignment: Optional[Assignment] = None) -> List[Assignment]:
    """Every solution the reference's DPLL returns, in the same order, each dict in
    the same insertion order.  Like REF.py:167 the caller's `assignment` dict is
    extended in place by the root's unit propagation."""
    init = None if assignment is None else [v if b else -v for v, b in assignment.items()]
    cap = 1024
    while True:
        r = dpll_batch([formula], mode="ref", max_solutions=0, sol_cap=cap,
                       inits=None if init is None else [init], time_limit=_time_limit)
        st = int(r.status[0])
        if st == _capi.DPLL_TIMEOUT:
            raise SolverTimeout(f"Timeout after {_time_limit:g} seconds")
        if st != _capi.DPLL_EXHAUSTED:
            raise _capi.SatmiError(f"dpll_optimized: GPU search ended with status {_capi.STATUS_NAMES.get(st, st)}")
        n = r.num_solutions(0)
        if n <= cap:
            break
        cap = n
    if assignment is not None:
        for lit in r.root_assignment(0)[len(init):]:
            assignment[abs(lit)] = lit > 0
    return [{abs(l): l > 0 for l in sol} for sol in r.solutions(0)]


def dpll_solve(formula: Formula):
    """Sound DPLL decision (same propagation / pure-literal / branching rules as
    REF.py's DPLL, decisions applied to the formula).  Returns (sat, model)."""
    r = dpll_batch([formula], mode="sound", max_solutions=1, time_limit=_time_limit)
    st = int(r.status[0])
    if st == _capi.DPLL_TIMEOUT:
        raise SolverTimeout(f"Timeout after {_time_limit:g} seconds")
    if r.num_solutions(0) > 0:
        return True, {abs(l): l > 0 for l in r.solutions(0)[0]}
    return False, None


def resolution_solver(formula: Formula) -> bool:
    from .resolution import resolution_solve
    return resolution_solve(formula, time_limit=_time_limit)


def davis_putnam_solver(formula: Formula) -> bool:
    from .dp import davis_putnam_solve
    return davis_putnam_solve(formula, time_limit=_time_limit)


def pysat_solver(formula: Formula) -> List[Assignment]:
    """REF.py:387-397 delegates to PySAT's Glucose3, a third-party library that
    is not part of this image.  It is used when installed; otherwise this raises."""
    try:
        from pysat.formula import CNF
        from pysat.solvers import Solver
    except ImportError as e:  # pragma: no cover - depends on the environment
        raise ImportError("pysat_solver needs the python-sat package (REF.py:6-7)") from e
    cnf = CNF()
    for clause in formula:
        cnf.append(clause)
    with Solver(name="glucose3", bootstrap_with=cnf) as solver:
        if solver.solve():
            return [{abs(lit): lit > 0 for lit in solver.get_model()}]
        return []


def cdcl_solve(formula: Formula) -> Tuple[bool, Optional[Assignment]]:
    """REF.py:382-384 on the GPU (csrc/cdcl.hip): the reference's CDCLSolver, same
    watch-list / dict / activity orders, so the same verdict and the same model
    dict.  The reference's loop can run forever; under the driver's deadline the
    call raises SolverTimeout like the other solvers."""
    from .cdcl import CdclLimit
    from .cdcl import cdcl_solve as _gpu_cdcl
    try:
        return _gpu_cdcl(formula, time_limit=_time_limit)
    except CdclLimit as e:
        raise SolverTimeout(f"Timeout after {_time_limit:g} seconds" if _time_limit else str(e)) from e


def hybrid_solver(formula: Formula, threshold=1000) -> List[Assignment]:
    """REF.py:400-404: PySAT above `threshold` clauses, DPLL below."""
    if len(formula) > threshold:
        return pysat_solver(formula)
    return dpll_optimized(formula)
