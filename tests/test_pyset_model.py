"""The CPython-3.10 set model (oracle/pyset.c) against the running interpreter.

The DP elimination order of the reference depends on CPython's set layout
(REF.py:100-103); the model is only trustworthy if it reproduces the real
interpreter's iteration order for the constructions the reference uses."""
import random
import sys

import pytest

import oracle

pytestmark = pytest.mark.skipif(sys.version_info[:2] != (3, 10), reason="model targets CPython 3.10")


def test_set_from_list_iteration_order():
    rng = random.Random(7)
    for _ in range(3000):
        n = rng.randint(0, 40)
        hi = rng.choice([4, 9, 20, 64, 300])
        keys = [rng.choice([-1, 1]) * rng.randint(1, hi) for _ in range(n)]
        assert oracle.pyset_from_list(keys) == list(set(keys)), keys


def test_resolvent_construction_order():
    rng = random.Random(11)
    for _ in range(3000):
        hi = rng.choice([5, 12, 40, 130])
        var = rng.randint(1, hi)
        a = [var] + [rng.choice([-1, 1]) * rng.randint(1, hi) for _ in range(rng.randint(0, 14))]
        b = [-var] + [rng.choice([-1, 1]) * rng.randint(1, hi) for _ in range(rng.randint(0, 14))]
        rng.shuffle(a)
        rng.shuffle(b)
        expect = list((set(a) - {var}) | (set(b) - {-var}))
        assert oracle.pyset_resolvent(a, var, b, -var) == expect, (a, b, var)


def test_variable_set_pop():
    rng = random.Random(3)
    for _ in range(2000):
        hi = rng.choice([6, 20, 70, 400])
        lists = [[rng.choice([-1, 1]) * rng.randint(1, hi) for _ in range(rng.randint(1, 6))]
                 for _ in range(rng.randint(1, 30))]
        sets = [set(c) for c in lists]
        variables = {abs(l) for c in sets for l in c}
        assert oracle.pyset_var_pop(lists) == variables.pop(), lists
