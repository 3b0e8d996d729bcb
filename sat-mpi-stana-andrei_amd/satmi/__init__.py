"""satmi -- MI355X-native clause-set solving (drop-in for the reference's solvers).

Layout:
    _capi.py      ctypes binding of libsatmi.so (include/satmi.h)
    cnf.py        CSR formula batches, generators, DIMACS
    dpll.py       batched DPLL (csrc/dpll.hip)
    solvers.py    the reference's solver entry points (same signatures)
"""
from . import _capi
from .cnf import CnfBatch, pack, uniform_ksat
from .dpll import DpllResult, dpll_batch

__all__ = ["CnfBatch", "pack", "uniform_ksat", "DpllResult", "dpll_batch", "_capi"]
