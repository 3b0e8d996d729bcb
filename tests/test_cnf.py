"""Host CSR containers (satmi/cnf.py): pack() round trips and its edge cases,
and menu_batch() draws formulas of generate_large_formula's shape (REF.py:21-29)."""
import random

import numpy as np
import pytest

from satmi import cnf, solvers


@pytest.mark.parametrize("formulas", [
    [], [[]], [[[1, -2]], [], [[3]], [[1], [2, 3, -1]]], [[[]], [[5]]], [[[-7, 2], []]],
])
def test_pack_round_trip_edges(formulas):
    b = cnf.pack(formulas)
    assert b.num_instances == len(formulas)
    assert [b.instance(i) for i in range(b.num_instances)] == formulas
    assert b.inst_nvars.tolist() == [max([abs(l) for c in f for l in c] + [0]) for f in formulas]
    assert b.inst_clause_begin.dtype == b.clause_lit_begin.dtype == b.lits.dtype == np.int32


def test_pack_round_trip_random_and_rejects_zero():
    random.seed(3)
    fs = [solvers.generate_large_formula(random.randint(0, 20), 4, 9) for _ in range(60)]
    b = cnf.pack(fs)
    assert [b.instance(i) for i in range(len(fs))] == fs
    with pytest.raises(ValueError):
        cnf.pack([[[1, 0]]])


def test_menu_batch_shape():
    b = cnf.menu_batch(300, 80, 3, 15, seed=7)
    assert b.num_instances == 300
    sizes = np.diff(b.clause_lit_begin)
    assert sizes.min() == 1 and sizes.max() == 3 and len(sizes) == 300 * 80
    for i in (0, 17, 299):
        f = b.instance(i)
        assert len(f) == 80
        assert all(len({abs(l) for l in c}) == len(c) and all(1 <= abs(l) <= 15 for l in c) for c in f)
    assert 0.4 < (b.lits < 0).mean() < 0.6
    assert (cnf.menu_batch(300, 80, 3, 15, seed=7).lits == b.lits).all()


def test_pack_rejects_out_of_range_and_accepts_iterables():
    """Literals beyond int32 are rejected, not wrapped; generators
    of formulas and of clauses pack like the lists they yield."""
    import pytest
    for bad in (2 ** 31, -(2 ** 31), 2 ** 40):
        with pytest.raises(ValueError):
            cnf.pack([[[1, bad]]])
    fs = [[[1, -2], [3]], [[-4, 5, 6]]]
    g = cnf.pack((iter(c) for c in f) for f in fs)
    b = cnf.pack(fs)
    assert [g.instance(i) for i in range(2)] == [b.instance(i) for i in range(2)] == fs
