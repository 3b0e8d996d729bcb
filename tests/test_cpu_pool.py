"""oracle/cpu_pool.py, the bench's CPU baseline pool (test infrastructure): the
set kinds solve every formula of the sample and cycle over it until the time
is up; the DPLL kind walks the sample once."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cpu_pool  # noqa: E402

from satmi import cnf  # noqa: E402


def _save(tmp_path, batch):
    for name, arr in (("icb", batch.inst_clause_begin), ("clb", batch.clause_lit_begin), ("lits", batch.lits)):
        np.save(os.path.join(tmp_path, name + ".npy"), np.ascontiguousarray(arr, dtype=np.int32))
    return str(tmp_path)


def test_set_kinds_cycle_over_the_sample(tmp_path):
    batch = cnf.uniform_ksat(3, 5, 30, 3, seed=4)
    path = _save(tmp_path, batch)
    for kind in ("dpset", "resset"):
        r = cpu_pool.run(kind, path, 0.3, 0, 2)
        assert r["kind"] == kind
        assert r["units"] > 3   # more than one pass over the 3 formulas
        assert r["units_per_s"] > 0


def test_dpll_kind_walks_the_sample_once(tmp_path):
    batch = cnf.uniform_ksat(5, 10, 42, 3, seed=9)
    r = cpu_pool.run("dpll", _save(tmp_path, batch), 30.0, 0, 2)
    assert r["units"] == 5
    assert r["unit_props"] > 0


def test_dpll_kind_with_more_workers_than_instances(tmp_path):
    """a worker past the sample's end solves nothing (it must not
    solve and count an instance another worker counted); an empty sample is
    no error."""
    batch = cnf.uniform_ksat(2, 10, 42, 3, seed=9)
    r = cpu_pool.run("dpll", _save(tmp_path, batch), 30.0, 0, 5)
    assert r["units"] == 2
    empty = tmp_path / "empty"
    empty.mkdir()
    for name, arr in (("icb", [0]), ("clb", [0]), ("lits", [0])):
        np.save(os.path.join(empty, name + ".npy"), np.asarray(arr, dtype=np.int32))
    assert cpu_pool.run("dpll", str(empty), 1.0, 0, 2)["units"] == 0
