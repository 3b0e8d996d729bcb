"""The Davis-Putnam pop fast path (csrc/dp.hip dp_pop_split_kernel, pyset_dev.h
py_size_after), checked against the live CPython interpreter (CPU only):
REF.py:100/:128 builds `{abs(lit) for clause in clauses for lit in clause}` and
pops it once; when every variable is below the table size the set reaches
after its distinct adds, each sits at its own slot whatever the insertion
order, so pop() returns the smallest -- the kernel then skips the sequential
set model.  Above that size the kernel keeps the model (tests/test_dp_gpu.py
covers both, sparse ids included)."""
import random
import sys

PY_MINSIZE = 8


def py_size_after(n):
    """Mirror of pyset_dev.h py_size_after."""
    mask = PY_MINSIZE - 1
    while True:
        thr = (mask * 3 + 4) // 5
        if n < thr:
            return mask + 1
        minused = thr * 2 if thr > 50000 else thr * 4
        ns = PY_MINSIZE
        while ns <= minused:
            ns <<= 1
        mask = ns - 1


def _table_slots(s):
    # sys.getsizeof(set) = the object + its table when the table is not the
    # small inline one; both grow in whole 16-B entries
    empty = sys.getsizeof(set())
    extra = sys.getsizeof(s) - empty
    return PY_MINSIZE if extra == 0 else extra // 16


def test_size_after_matches_the_interpreter():
    for n in list(range(0, 200)) + [1000, 4095, 20000, 60000]:
        s = set()
        for v in range(1, n + 1):
            s.add(v)
        assert _table_slots(s) == py_size_after(n), n


def test_pop_is_the_smallest_below_the_table_size():
    rng = random.Random(5)
    checked = 0
    for _ in range(3000):
        n = rng.randint(1, 120)
        size = py_size_after(n)
        vals = rng.sample(range(1, size), min(n, size - 1))
        lits = [v if rng.random() < 0.5 else -v for v in vals for _ in range(rng.randint(1, 3))]
        rng.shuffle(lits)
        s = {abs(x) for x in lits}   # the reference's construction
        if max(s) < py_size_after(len(s)):
            assert s.pop() == min(vals)
            checked += 1
    assert checked > 1000


def test_sparse_ids_need_the_model():
    # above the table size the insertion order decides: the fast path must not apply
    s = {abs(x) for x in [37 * 9, 37, 37 * 5]}
    assert max(s) >= py_size_after(len(s))
