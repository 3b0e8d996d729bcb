"""GPU parity of the batched DPLL kernel (csrc/dpll.hip) through the C ABI.

REF mode against the reference's own outputs (tests/golden/dpll_ref.json);
SOUND mode against the CPU oracle (counters and models, bit-exact) and against
the reference's Davis-Putnam verdicts; full-size batches through
size-independent properties (every model satisfies every clause, verdicts
agree with the oracle on a sample)."""
import json
import os
import random

import numpy as np
import pytest

import oracle
from satmi import _capi, cnf
from satmi.dpll import dpll_batch

pytestmark = pytest.mark.gpu

CTR = ("nodes", "decisions", "unit_props", "pure_assigns", "conflicts", "solutions")


def _golden(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as fh:
        return json.load(fh)["cases"]


def _satisfies(formula, model_lits):
    model = {abs(l): l > 0 for l in model_lits}
    return all(any(model.get(abs(l)) == (l > 0) for l in c) for c in formula)


def test_ref_mode_matches_reference_golden(golden_dir):
    cases = _golden(golden_dir, "dpll_ref.json")
    fs = [c["formula"] for c in cases]
    inits = [c["init"] for c in cases]
    cap = max(len(c["solutions"]) for c in cases) + 1
    r = dpll_batch(fs, mode="ref", max_solutions=0, sol_cap=cap, inits=inits, time_limit=20.0)
    for b, c in enumerate(cases):
        assert r.status[b] == _capi.DPLL_EXHAUSTED, c["formula"]
        assert r.solutions(b) == c["solutions"], c["formula"]
        got = r.counter_dict(b)
        for k, v in c["counters"].items():
            assert got[k] == v, (k, c["formula"])
        if "init_after" in c:
            assert r.root_assignment(b) == c["init_after"]


def test_sound_mode_matches_oracle_small():
    rng = random.Random(5)
    fs = []
    for i in range(300):
        n = rng.randint(3, 14)
        m = rng.randint(1, 70)
        k = rng.randint(1, 5)
        f = [[v if rng.random() < 0.5 else -v for v in rng.sample(range(1, n + 1), min(k, n) if i % 3 else rng.randint(1, min(k, n)))]
             for _ in range(m)]
        fs.append(f)
    for mode, maxs in (("sound", 1), ("sound", 0), ("ref", 0)):
        r = dpll_batch(fs, mode=mode, max_solutions=maxs, sol_cap=64, time_limit=20.0)
        for b, f in enumerate(fs):
            o = oracle.dpll(f, mode, max_solutions=maxs, sol_cap=64)
            got = r.counter_dict(b)
            for k in CTR:
                assert got[k] == o["counters"][k], (mode, k, f)
            assert r.solutions(b) == o["solutions"][:64], (mode, f)


def test_sound_verdicts_match_reference_dp(golden_dir):
    cases = [c for c in _golden(golden_dir, "dp_ref.json") if all(len(cl) for cl in c["formula"])]
    fs = [c["formula"] for c in cases]
    r = dpll_batch(fs, mode="sound", max_solutions=1, time_limit=20.0)
    for b, c in enumerate(cases):
        sat = r.num_solutions(b) > 0
        assert sat == c["result"], c["formula"]
        if sat:
            assert _satisfies(c["formula"], r.solutions(b)[0])


@pytest.mark.parametrize("n,k,alpha,B", [(50, 3, 4.26, 4096), (100, 3, 4.26, 2048)])
def test_full_size_properties(n, k, alpha, B):
    m = int(round(alpha * n))
    batch = cnf.uniform_ksat(B, n, m, k, seed=n * 7 + k)
    r = dpll_batch(batch, mode="sound", max_solutions=1, time_limit=60.0)
    assert ((r.status == _capi.DPLL_STOPPED) | (r.status == _capi.DPLL_EXHAUSTED)).all()
    nsat = 0
    for b in range(B):
        if r.num_solutions(b):
            nsat += 1
            assert _satisfies(batch.instance(b), r.solutions(b)[0])
        else:
            assert r.status[b] == _capi.DPLL_EXHAUSTED
    assert 0 < nsat < B or k == 5
    # bit-exact against the oracle on a sample
    for b in range(0, B, max(1, B // 12))[:12]:
        o = oracle.dpll(batch.instance(b), "sound", max_solutions=1, sol_cap=1)
        got = r.counter_dict(b)
        for key in CTR:
            assert got[key] == o["counters"][key], (b, key)
        assert r.solutions(b)[:1] == o["solutions"][:1]


def test_edge_cases():
    fs = [[], [[]], [[1]], [[1], [-1]], [[1, -1]], [[3, -3, 2]], [[1, 2], [], [3]], [[7]]]
    for mode in ("ref", "sound"):
        r = dpll_batch(fs, mode=mode, max_solutions=0, sol_cap=16, time_limit=20.0)
        for b, f in enumerate(fs):
            o = oracle.dpll(f, mode, sol_cap=16)
            assert r.solutions(b) == o["solutions"]
            for key in CTR:
                assert r.counter_dict(b)[key] == o["counters"][key]


def test_limits_and_too_large():
    f = cnf.uniform_ksat(1, 40, 170, 3, seed=1).instance(0)
    o = oracle.dpll(f, "ref", node_limit=50, sol_cap=4)
    assert o["status"] == 2
    r = dpll_batch([f], mode="ref", max_solutions=0, node_limit=50, sol_cap=4)
    assert r.status[0] == _capi.DPLL_NODE_LIMIT
    assert r.counter_dict(0)["nodes"] == 51
    hard = cnf.uniform_ksat(1, 250, 1065, 3, seed=3).instance(0)
    r = dpll_batch([hard], mode="sound", max_solutions=0, time_limit=0.05, sol_cap=4)
    assert r.status[0] == _capi.DPLL_TIMEOUT
