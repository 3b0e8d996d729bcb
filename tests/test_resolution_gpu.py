"""GPU parity of resolution saturation (csrc/resolution.hip) through the C ABI:
verdicts and the exact set of clauses every pass adds, against the reference's
own outputs (tests/golden/resolution_ref.json) and the CPU oracle."""
import json
import os
import random

import pytest

import oracle
from conftest import clause_set_sha
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


def test_pigeonhole_php43_four_passes(golden_dir):
    """The bench workload itself (bench.py --workload php-res): the first four
    passes of PHP(4,3) -- the 4th resolves 27.8 M pairs and adds 163,954
    clauses -- add exactly the clause SETS the reference's own
    resolution_solver adds (tests/golden/resolution_php43.json,
    make_golden_bench.py): passes 1-3 clause by clause, pass 4 by size and
    sha256 of the canonical set."""
    with open(os.path.join(golden_dir, "resolution_php43.json")) as fh:
        (c,) = json.load(fh)["cases"]
    f = cnf.pigeonhole(3)
    assert f == c["formula"]
    r = resolve(f, max_passes=4, record=True)
    assert r["result"] == -1 and r["passes"] == 4
    assert r["pass_new"] == [p["count"] for p in c["passes"]] == [36, 270, 7132, 163954]
    for k, p in enumerate(c["passes"]):
        assert clause_set_sha(r["clauses"][k]) == p["sha256"], k
        if "clauses" in p:
            assert r["clauses"][k] == p["clauses"], k


def test_repeated_calls_replay_the_captured_segment(golden_dir):
    """A call's first segment (state init, packing, seeding, the first batch of
    passes) is captured into a HIP graph the second time it repeats and
    replayed after (csrc/resolution.hip ResGraph): the bench's php-res call
    five times in a row, with other formulas in between (a new key: the
    segment is re-captured), adds the reference's sets every time."""
    with open(os.path.join(golden_dir, "resolution_php43.json")) as fh:
        (c,) = json.load(fh)["cases"]
    f = cnf.pigeonhole(3)
    want = [p["count"] for p in c["passes"]]
    for k in range(5):
        r = resolve(f, max_passes=4, record=k == 4)
        assert r["result"] == -1 and r["pass_new"] == want, k
        if k == 2:   # another formula in between, twice (captured on its second call)
            g = cnf.pigeonhole(2)
            o = oracle.resolution(g)
            for _ in range(2):
                rg = resolve(g)
                assert (rg["result"], rg["pass_new"]) == (o["result"], o["pass_new"])
    for k, p in enumerate(c["passes"]):   # the last call recorded its sets
        assert clause_set_sha(r["clauses"][k]) == p["sha256"], k


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
    """PHP(5,4) saturates through passes far beyond a second (its 5th pass
    resolves ~10^11 pairs): the deadline, read by every workgroup before each
    clause j, stops the saturation as a timeout (result -1) within the limit,
    after the passes the oracle reproduces."""
    import time
    f = cnf.pigeonhole(4)
    o = oracle.resolution(f, max_passes=3)
    t = time.perf_counter()
    r = resolve(f, time_limit=0.3)
    dt = time.perf_counter() - t
    assert r["result"] == -1 and r["passes"] >= 3, r
    assert r["pass_new"][:3] == o["pass_new"]
    assert dt < 5.0, dt


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


def test_candidate_buffer_rerun_path():
    """Beyond 31 variables a chunk's candidates go through a buffer capped at
    1 GiB; a chunk that overflows it is re-run at its counted size (ADVICE
    r03).  With the cap shrunk to 4 KiB (test knob) every sizeable chunk takes
    that path and the passes still add exactly the oracle's clause sets."""
    from satmi import _capi
    L = _capi.load()
    rng = random.Random(40)
    nvars = 40
    vs = list(range(1, nvars + 1))
    rng.shuffle(vs)
    f = [[v if rng.random() < 0.5 else -v for v in vs[i:i + 3]] for i in range(0, nvars, 3)]
    f += [[v if rng.random() < 0.5 else -v for v in rng.sample(vs, 2)] for _ in range(30)]
    o = oracle.resolution(f, record=True, max_passes=3)
    _capi.check(L.satmi_resolution_debug_cand_bytes(4096), "cand bytes")
    try:
        r = resolve(f, record=True, max_passes=3)
    finally:
        _capi.check(L.satmi_resolution_debug_cand_bytes(0), "cand bytes reset")
    assert sum(o["pass_new"]) * 16 > 4096   # the candidates do not fit the shrunk buffer
    assert r["result"] == o["result"] and r["pass_new"] == o["pass_new"]
    assert [sorted(p) for p in r["clauses"]] == [sorted(p) for p in o["clauses"]]



def test_graph_replay_alternating_formulas_of_one_shape():
    """the captured segment is keyed by clause count, buffers,
    table size and argument bytes, not by the clauses.  Two different formulas
    with the same clause count and variable count (<= 31: the packed path),
    alternated so both are captured and replayed several times, must each add
    their own clause sets every call (a replay reads the newly encoded clauses)."""
    rng = random.Random(55)
    nv, m = 9, 14
    fs = []
    while len(fs) < 2:
        f = [sorted(rng.sample(range(1, nv + 1), 3)) for _ in range(m)]
        f = [[v if rng.random() < 0.5 else -v for v in c] for c in f]
        if len({abs(l) for c in f for l in c}) == nv and f not in fs:
            fs.append(f)
    want = [oracle.resolution(f, record=True, max_passes=3) for f in fs]
    assert want[0]["pass_new"] != want[1]["pass_new"] or want[0]["clauses"] != want[1]["clauses"]
    for k in range(8):
        i = k % 2
        r = resolve(fs[i], max_passes=3, record=True)
        assert (r["result"], r["pass_new"]) == (want[i]["result"], want[i]["pass_new"]), (k, i)
        assert [sorted(p) for p in r["clauses"]] == [sorted(p) for p in want[i]["clauses"]], (k, i)


def test_regrowth_call_reports_each_pass_once():
    """a pass stopped by an overflow runs again on regrown
    buffers; its candidates and kernel time count once.  A call on fresh
    (trimmed) workspaces regrows during PHP(4,3)'s 4th pass; its statistics
    equal those of the next call, which needs no regrowth."""
    from satmi import _capi
    from satmi.resolution import last_stats
    f = cnf.pigeonhole(3)
    _capi.trim_workspaces()
    r1 = resolve(f, max_passes=4)
    s1 = last_stats()
    r2 = resolve(f, max_passes=4)
    s2 = last_stats()
    assert r1 == r2
    assert (s1["pairs"], s1["candidates"]) == (s2["pairs"], s2["candidates"])
    assert s1["pair_ms"] < 1.6 * s2["pair_ms"] + 0.05


def test_bench_random_unsat_set_matches_oracle():
    """The bench's configs[3] `rand-res` set (16 random 3-SAT formulas n=7,
    m=49, seed 7001): the first two, every pass's clause set against the oracle."""
    batch = cnf.uniform_ksat(16, 7, 49, 3, seed=7001)
    for b in (0, 1):
        f = batch.instance(b)
        o = oracle.resolution(f, record=True)
        r = resolve(f, record=True, time_limit=60.0)
        assert r["result"] == o["result"]
        assert list(r["pass_new"]) == list(o["pass_new"])
        assert [sorted(p) for p in r["clauses"]] == [sorted(p) for p in o["clauses"]]


def test_general_then_packed_calls_share_the_table():
    """the general path (> 31 variables) fills the workspace's
    table with clause indices; the next packed call (<= 31 variables) on the
    same thread reuses that table and must empty it first.  A stale index i
    equals the packed key of the all-positive clause over dense variables
    bit-set i, so the packed formulas here are full of small all-positive
    clauses; every call's passes must equal the oracle's."""
    from satmi import _capi
    rng = random.Random(71)
    nvars = 40
    vs = list(range(1, nvars + 1))
    big = [[v if rng.random() < 0.5 else -v for v in vs[i:i + 3]] for i in range(0, nvars, 3)]
    big += [[v if rng.random() < 0.5 else -v for v in rng.sample(vs, 2)] for _ in range(30)]
    small = [
        [[1, 2], [1], [2], [1, 3], [-1, -2, 3], [-3, 4], [-4]],
        [[1, 2], [2, 3], [1, 3], [-1, -2], [-2, -3], [-1, -3], [1, 2, 3]],
        [[1], [2], [1, 2], [3], [1, 3], [2, 3], [1, 2, 3], [-1, -2, -3]],
    ]
    want_big = oracle.resolution(big, record=True, max_passes=2)
    want = [oracle.resolution(f, record=True) for f in small]
    _capi.trim_workspaces()
    for k in range(6):
        f, w = small[k % 3], want[k % 3]
        r = resolve(f, record=True)
        assert (r["result"], r["pass_new"]) == (w["result"], w["pass_new"]), (k, f)
        assert [sorted(p) for p in r["clauses"]] == [sorted(p) for p in w["clauses"]], (k, f)
        rb = resolve(big, record=True, max_passes=2)
        assert (rb["result"], rb["pass_new"]) == (want_big["result"], want_big["pass_new"]), k
