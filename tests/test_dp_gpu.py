"""GPU parity of Davis-Putnam elimination (csrc/dp.hip) through the C ABI: the
eliminated variables (CPython's set.pop() order, modelled on the device) and
every intermediate clause list -- each clause in its Python set iteration
order -- against the reference's own outputs (tests/golden/dp_ref.json) and
the CPU oracle."""
import json
import os
import random

import pytest

import oracle
from conftest import clause_list_sha
from satmi import cnf
from satmi.dp import eliminate

pytestmark = pytest.mark.gpu


def _cases(golden_dir):
    with open(os.path.join(golden_dir, "dp_ref.json")) as fh:
        return json.load(fh)["cases"]


def test_matches_reference_golden(golden_dir):
    for c in _cases(golden_dir):
        r = eliminate(c["formula"], record=True, time_limit=60.0)
        assert r["result"] == int(c["result"]), c["formula"]
        assert r["vars"] == [s["var"] for s in c["steps"]], c["formula"]
        for k, s in enumerate(c["steps"]):
            if "clauses" in s:
                assert r["clauses"][k] == s["clauses"], (c["formula"], k)


def _completed(o):
    return o["steps"] if o["result"] == 1 else max(o["steps"] - 1, 0)


def test_matches_oracle_random():
    rng = random.Random(29)
    for it in range(120):
        n = rng.randint(2, 12)
        m = rng.randint(1, 30)
        f = [[v if rng.random() < 0.5 else -v for v in rng.sample(range(1, n + 1), rng.randint(1, min(4, n)))]
             for _ in range(m)]
        if it % 9 == 0:
            f.append([1, -1] + ([2] if n > 1 else []))      # tautological clause: in the pos and neg lists
        if it % 5 == 0:
            f.append(list(f[0]))                             # duplicate clause
        if it % 4 == 1:
            f = [[x * 37 for x in c] for c in f]             # sparse ids: collisions in the set tables
        if it % 7 == 3:
            f = [c + [c[0]] for c in f]                      # duplicate literals inside clauses
        o = oracle.dp(f, record=True)
        r = eliminate(f, record=True, time_limit=60.0)
        assert r["result"] == o["result"], f
        assert r["vars"] == o["vars"], f
        assert r["clauses"] == o["clauses"][:_completed(o)], f


def test_edge_cases_and_pigeonhole():
    for f in ([], [[]], [[1]], [[1], [-1]], [[1, -1]], [[1, 1], [-1]], [[1, 2], [], [-1]],
              cnf.pigeonhole(2), cnf.pigeonhole(3)):
        o = oracle.dp(f, record=True)
        r = eliminate(f, record=True)
        assert (r["result"], r["vars"]) == (o["result"], o["vars"]), f
        assert r["clauses"] == o["clauses"][:_completed(o)], f


def test_limits():
    f = cnf.uniform_ksat(1, 14, 60, 3, seed=9).instance(0)
    o = oracle.dp(f, step_limit=2)
    r = eliminate(f, step_limit=2)
    assert (r["result"], r["vars"]) == (o["result"], o["vars"]) and r["result"] == -1
    o = oracle.dp(f, clause_limit=70)
    r = eliminate(f, clause_limit=70)
    assert (r["result"], r["vars"]) == (o["result"], o["vars"])


def test_php65_every_step_matches_oracle():
    """The configs[3] bench formula PHP(6,5) (bench.py --workload php-dp): the
    30 eliminated variables and all 29 intermediate clause lists (26,693
    clauses, each in its set iteration order) equal the oracle's, and the
    verdict is False (REF.py:117-118)."""
    f = cnf.pigeonhole(5)
    o = oracle.dp(f, record=True, rec_cap=1 << 22)
    r = eliminate(f, record=True)
    assert r["result"] == o["result"] == 0
    assert r["vars"] == o["vars"] and len(r["vars"]) == 30
    assert r["clauses"] == o["clauses"][:_completed(o)]


def test_php65_matches_reference_fixture(golden_dir):
    """The same workload against the reference itself: the reference's own
    davis_putnam_solver on PHP(6,5) (tests/golden/dp_php65.json,
    make_golden_bench.py) -- the eliminated variables, the verdict, and every
    intermediate clause list (clause order and each clause's set iteration
    order) by length and sha256, the first four in full."""
    with open(os.path.join(golden_dir, "dp_php65.json")) as fh:
        (c,) = json.load(fh)["cases"]
    r = eliminate(c["formula"], record=True)
    assert r["result"] == int(c["result"]) == 0
    assert r["vars"] == [s["var"] for s in c["steps"]]
    done = [s for s in c["steps"] if "sha256" in s]
    assert len(r["clauses"]) == len(done) == 29
    for k, s in enumerate(done):
        assert len(r["clauses"][k]) == s["n"], k
        assert clause_list_sha(r["clauses"][k]) == s["sha256"], k
        if "clauses" in s:
            assert r["clauses"][k] == s["clauses"], k
    # the same solve without recording (the bench path: one wait per batch)
    r2 = eliminate(c["formula"])
    assert (r2["result"], r2["vars"]) == (r["result"], r["vars"])


def test_concurrent_solves_from_threads():
    """satmi_dp_host from several host threads at once (each on its own stream
    and buffers, as bench.py --threads runs it): every solve equals the oracle."""
    from concurrent.futures import ThreadPoolExecutor
    fs = [cnf.pigeonhole(4), cnf.pigeonhole(3)] + [cnf.uniform_ksat(1, 12, 50, 3, seed=s).instance(0)
                                                   for s in range(6)]
    want = [oracle.dp(f, record=True) for f in fs]
    with ThreadPoolExecutor(4) as ex:
        for _ in range(3):
            got = list(ex.map(lambda f: eliminate(f, record=True), fs))
            for f, o, r in zip(fs, want, got):
                assert (r["result"], r["vars"]) == (o["result"], o["vars"]), f
                assert r["clauses"] == o["clauses"][:_completed(o)], f
    # the pooled workspaces freed, the next solves allocate afresh
    from satmi import _capi
    _capi.trim_workspaces()
    for f, o in zip(fs[:2], want[:2]):
        r = eliminate(f, record=True)
        assert (r["result"], r["vars"]) == (o["result"], o["vars"]) and r["clauses"] == o["clauses"][:_completed(o)]


def test_bench_random_unsat_set_matches_oracle():
    """The bench's configs[3] `rand-dp` set (16 random 3-SAT formulas n=16,
    m=96, seed 7002): verdicts, eliminated variables and every clause list."""
    batch = cnf.uniform_ksat(16, 16, 96, 3, seed=7002)
    unsat = 0
    for b in range(16):
        f = batch.instance(b)
        o = oracle.dp(f, record=True)
        r = eliminate(f, record=True, time_limit=60.0)
        assert r["result"] == o["result"], b
        assert r["vars"] == o["vars"], b
        assert r["clauses"] == o["clauses"][:_completed(o)], b
        unsat += r["result"] == 0
    assert unsat >= 12   # past the threshold: the set is mostly UNSAT


def test_launch_chain_floor():
    """satmi_launch_chain_floor (the php-dp roofline's peak): an empty chain of
    dependent one-block launches replayed from a HIP graph takes a positive,
    microsecond-scale time per launch, and no less per launch than a solve's
    real kernels (which do work)."""
    from satmi import _capi
    from satmi.dp import last_stats
    floor = _capi.launch_chain_floor(280, reps=5)
    assert 0.05 < floor < 50.0
    eliminate(cnf.pigeonhole(5))
    st = last_stats()
    assert st["device_ms"] * 1e3 / st["launches"] >= floor
    with pytest.raises(_capi.SatmiError):
        _capi.launch_chain_floor(0)


@pytest.fixture
def dp_inline(monkeypatch):
    """The opt-in inline-step form of the pop kernel (SATMI_DP_INLINE=1: small
    steps run to their end inside one workgroup; read per call)."""
    monkeypatch.setenv("SATMI_DP_INLINE", "1")
    yield


def test_inline_steps_match_reference_fixture_and_oracle(golden_dir, dp_inline):
    """The inline-step form (csrc/dp.hip "Inline steps") gives the pipeline's
    results exactly: PHP(6,5) against the reference's own run, step by step
    (recording runs one step per slot, inline when it fits) and unrecorded
    (many inline steps per slot, the assembly of large ones handed to the
    pipeline's assemble kernel), and random formulas against the oracle."""
    with open(os.path.join(golden_dir, "dp_php65.json")) as fh:
        (c,) = json.load(fh)["cases"]
    r = eliminate(c["formula"], record=True)
    assert r["result"] == int(c["result"]) == 0
    assert r["vars"] == [s["var"] for s in c["steps"]]
    done = [s for s in c["steps"] if "sha256" in s]
    for k, s in enumerate(done):
        assert clause_list_sha(r["clauses"][k]) == s["sha256"], k
    for _ in range(3):   # the learned slot count and the captured graph replayed
        r2 = eliminate(c["formula"])
        assert (r2["result"], r2["vars"]) == (r["result"], r["vars"])
    rng = random.Random(31)
    for it in range(60):
        n = rng.randint(2, 12)
        m = rng.randint(1, 30)
        f = [[v if rng.random() < 0.5 else -v for v in rng.sample(range(1, n + 1), rng.randint(1, min(4, n)))]
             for _ in range(m)]
        if it % 4 == 1:
            f = [[x * 37 for x in c] for c in f]
        o = oracle.dp(f, record=True)
        r = eliminate(f, record=True, time_limit=60.0)
        assert (r["result"], r["vars"]) == (o["result"], o["vars"]), f
        assert r["clauses"] == o["clauses"][:_completed(o)], f
        r2 = eliminate(f)
        assert (r2["result"], r2["vars"]) == (o["result"], o["vars"]), f
    batch = cnf.uniform_ksat(16, 16, 96, 3, seed=7002)   # the bench's rand-dp set
    for b in range(16):
        f = batch.instance(b)
        o = oracle.dp(f)
        assert (lambda x: (x["result"], x["vars"]))(eliminate(f)) == (o["result"], o["vars"]), b
