"""GPU parity of resolution saturation (csrc/resolution.hip) through the C ABI:
verdicts and the exact set of clauses every pass adds, against the reference's
own outputs (tests/golden/resolution_ref.json) and the CPU oracle."""
import json
import os
import random

import pytest

import oracle
from satmi import cnf
from satmi.resolution import resolve

pytestmark = pytest.mark.gpu


def _cases(golden_dir):
    with open(os.path.join(golden_dir, "resolution_ref.json")) as fh:
        return json.load(fh)["cases"]


def test_matches_reference_golden(golden_dir):
    for c in _cases(golden_dir):
        r = resolve(c["formula"], record=True, time_limit=60.0)
        assert r["result"] == int(c["result"]), c["formula"]
        got = [sorted(p) for p in r["clauses"]]
        assert got == [sorted(sorted(x) for x in p) for p in c["passes"]], c["formula"]


def test_matches_oracle_random():
    rng = random.Random(17)
    for it in range(60):
        n = rng.randint(2, 7)
        m = rng.randint(1, 12)
        f = [[v if rng.random() < 0.5 else -v for v in rng.sample(range(1, n + 1), rng.randint(1, min(3, n)))]
             for _ in range(m)]
        if it % 7 == 0:
            f.append(list(f[0]))                      # duplicate clause
        if it % 11 == 0:
            f.append([1, -1, 2][:min(3, n + 1)])      # tautological input clause
        o = oracle.resolution(f, record=True)
        r = resolve(f, record=True, time_limit=60.0)
        assert r["result"] == o["result"], f
        assert [sorted(p) for p in r["clauses"]] == [sorted(p) for p in o["clauses"]], f


def test_edge_cases():
    for f, want in (([], 1), ([[]], 1), ([[1]], 1), ([[1], [-1]], 0), ([[1, -1]], 1), ([[1, 1], [-1]], 0),
                    ([[1, 2], [], [-1]], 1)):
        o = oracle.resolution(f)
        r = resolve(f)
        assert r["result"] == o["result"] == want, f


def test_pigeonhole_and_limits():
    f = cnf.pigeonhole(2)
    assert resolve(f)["result"] == 0
    r = resolve(cnf.uniform_ksat(1, 8, 20, 3, seed=3).instance(0), max_passes=1)
    o = oracle.resolution(cnf.uniform_ksat(1, 8, 20, 3, seed=3).instance(0), max_passes=1)
    assert r["passes"] <= 1 and r["pass_new"][:1] == o["pass_new"][:1]


def test_pigeonhole_php43_four_passes():
    """A mid-size saturation (bench.py --workload php-res): the first four
    passes of PHP(4,3) -- the 4th resolves 27.8 M pairs and adds 163,954
    clauses -- add exactly the oracle's clause counts."""
    f = cnf.pigeonhole(3)
    r = resolve(f, max_passes=4)
    assert r["result"] == -1 and r["passes"] == 4
    assert r["pass_new"] == [36, 270, 7132, 163954]


@pytest.mark.parametrize("base", [(1 << 31) - 37, (1 << 32) - 50])
def test_append_slots_past_2_31(base):
    """The pair kernel's candidate slots start at `base` (test knob): the first
    passes of PHP(4,3) write slots across 2^31 / 2^32 (the 64-bit slot
    broadcast and the dedup's int64 candidate indices) and must add exactly
    the oracle's clause sets."""
    from satmi import _capi
    L = _capi.load()
    f = cnf.pigeonhole(3)
    o = oracle.resolution(f, record=True, max_passes=3)
    _capi.check(L.satmi_resolution_debug_slot_base(base), "slot base")
    try:
        r = resolve(f, record=True, max_passes=3)
    finally:
        _capi.check(L.satmi_resolution_debug_slot_base(0), "slot base reset")
    assert sum(r["pass_new"]) > 7000
    assert r["result"] == o["result"] and r["pass_new"] == o["pass_new"]
    assert [sorted(p) for p in r["clauses"]] == [sorted(p) for p in o["clauses"]]


def test_deadline_inside_a_pass():
    """PHP(4,3) saturates through passes of 1.5e10 pairs and more (pass 6 and
    on), run in chunks of 2^27 pairs with the deadline checked between them:
    the saturation stops as a timeout (result -1) within a chunk of the
    limit, after at least the passes the oracle-checked test above covers."""
    import time
    t = time.perf_counter()
    r = resolve(cnf.pigeonhole(3), time_limit=0.5)
    dt = time.perf_counter() - t
    assert r["result"] == -1 and r["passes"] >= 4, r
    assert r["pass_new"][:4] == [36, 270, 7132, 163954]
    assert dt < 10.0, dt


@pytest.mark.parametrize("nvars", [31, 32, 33, 70])
def test_table_forms_around_31_variables(nvars):
    """Up to 31 distinct variables the dedup table holds packed keys (one word,
    compared in register); beyond, clause / candidate indices whose keys are
    compared in memory (and 2 words per sign past 64).  Both forms add exactly
    the oracle's clause sets, on formulas that use every variable."""
    rng = random.Random(nvars)
    for _ in range(4):
        vs = list(range(1, nvars + 1))
        rng.shuffle(vs)
        f = [[v if rng.random() < 0.5 else -v for v in vs[i:i + 3]] for i in range(0, nvars, 3)]
        f += [[v if rng.random() < 0.5 else -v for v in rng.sample(range(1, nvars + 1), 2)] for _ in range(nvars // 2)]
        o = oracle.resolution(f, record=True, max_passes=3)
        r = resolve(f, record=True, max_passes=3)
        assert r["result"] == o["result"] and r["pass_new"] == o["pass_new"], f
        assert [sorted(p) for p in r["clauses"]] == [sorted(p) for p in o["clauses"]], f
