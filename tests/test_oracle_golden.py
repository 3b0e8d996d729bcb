"""Pin the CPU oracle against the reference's own outputs (tests/golden/*.json,
produced by tests/golden/make_golden.py running the reference functions)."""
import json
import os

import pytest

import oracle
from conftest import clause_list_sha, clause_set_sha


def _load(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as fh:
        return json.load(fh)["cases"]


def test_dpll_ref_mode_matches_reference(golden_dir):
    cases = _load(golden_dir, "dpll_ref.json")
    assert len(cases) > 50
    for c in cases:
        r = oracle.dpll(c["formula"], "ref", init=c["init"])
        assert r["status"] == 0
        assert r["solutions"] == c["solutions"], c["formula"]
        for k, v in c["counters"].items():
            assert r["counters"][k] == v, (k, c["formula"])
        if "init_after" in c:
            assert r["root_assign"] == c["init_after"]


def test_dp_matches_reference_steps(golden_dir):
    cases = _load(golden_dir, "dp_ref.json")
    assert len(cases) > 50
    for c in cases:
        r = oracle.dp(c["formula"], record=True)
        assert r["result"] == int(c["result"])
        assert r["vars"] == [s["var"] for s in c["steps"]]
        for k, s in enumerate(c["steps"]):
            if "clauses" in s:
                assert r["clauses"][k] == s["clauses"]


def test_resolution_matches_reference_passes(golden_dir):
    cases = _load(golden_dir, "resolution_ref.json")
    for c in cases:
        r = oracle.resolution(c["formula"], record=True)
        assert r["result"] == int(c["result"])
        assert r["clauses"] == c["passes"]


def test_dp_php65_matches_reference_every_step(golden_dir):
    """The configs[3] `php-dp` bench formula at full size: the oracle against
    the reference's own davis_putnam_solver on PHP(6,5)
    (tests/golden/dp_php65.json, make_golden_bench.py) -- the 30 eliminated
    variables, the verdict, and every one of the 29 intermediate clause lists
    (each clause in its set iteration order) by length and sha256, the first
    four in full."""
    (c,) = _load(golden_dir, "dp_php65.json")
    r = oracle.dp(c["formula"], record=True, rec_cap=1 << 22)
    assert r["result"] == int(c["result"]) == 0
    assert r["vars"] == [s["var"] for s in c["steps"]] and len(r["vars"]) == 30
    done = [s for s in c["steps"] if "sha256" in s]
    assert len(done) == 29 and len(r["clauses"]) == 29
    for k, s in enumerate(done):
        assert len(r["clauses"][k]) == s["n"], k
        assert sum(len(x) for x in r["clauses"][k]) == s["lits"], k
        assert clause_list_sha(r["clauses"][k]) == s["sha256"], k
        if "clauses" in s:
            assert r["clauses"][k] == s["clauses"], k


def test_resolution_php43_matches_reference_four_passes(golden_dir):
    """The configs[3] `php-res` bench workload at full size: the oracle's
    new-clause SET of each of the first four saturation passes of PHP(4,3)
    equals the reference's own resolution_solver's (tests/golden/
    resolution_php43.json, make_golden_bench.py): passes 1-3 clause by clause,
    pass 4 (163,954 clauses) by size and sha256 of the canonical set."""
    (c,) = _load(golden_dir, "resolution_php43.json")
    r = oracle.resolution(c["formula"], record=True, max_passes=4, rec_cap=1 << 23)
    assert r["result"] == -1 and r["passes"] == 4
    assert r["pass_new"] == [p["count"] for p in c["passes"]] == [36, 270, 7132, 163954]
    for k, p in enumerate(c["passes"]):
        assert clause_set_sha(r["clauses"][k]) == p["sha256"], k
        if "clauses" in p:
            assert sorted(sorted(x) for x in r["clauses"][k]) == p["clauses"], k


def test_sound_mode_verdicts_match_reference_dp(golden_dir):
    """SOUND DPLL (decisions applied as unit clauses) is a complete decision
    procedure: its verdict must equal the reference Davis-Putnam verdict, and
    every model it returns must satisfy every clause."""
    cases = _load(golden_dir, "dp_ref.json")
    for c in cases:
        f = c["formula"]
        r = oracle.dpll(f, "sound", max_solutions=1)
        sat = r["counters"]["solutions"] > 0
        if any(len(cl) == 0 for cl in f):
            continue  # REF.py treats an input empty clause specially in both solvers
        assert sat == c["result"], f
        if sat:
            model = {abs(l): l > 0 for l in r["solutions"][0]}
            for cl in f:
                assert any(model.get(abs(l)) == (l > 0) for l in cl), (f, cl)


SOUND_CTR = ("nodes", "decisions", "unit_props", "pure_assigns", "conflicts")


def test_sound_mode_matches_reference_rewritten_branch(golden_dir):
    """The benchmarked SOUND semantics, pinned to the reference's own code:
    tests/golden/dpll_sound_ref.json comes from REF.py's dpll_optimized with
    only the branch statements of REF.py:210-213 rewritten (the branch literal
    recursed on as the unit clause `formula + [[lit]]`; make_golden_sound.py).
    Every counter and the first model at the first-model stop (the bench's
    max_solutions=1), and the full enumeration where the reference finished."""
    cases = _load(golden_dir, "dpll_sound_ref.json")
    tags = {c["tag"] for c in cases}
    assert {"edge", "generator", "configs1_n50", "configs2_n100"} <= tags
    assert sum(c["tag"] == "configs2_n100" for c in cases) >= 48
    for c in cases:
        f = c["formula"]
        r = oracle.dpll(f, "sound", max_solutions=1, sol_cap=1)
        for k in SOUND_CTR:
            assert r["counters"][k] == c["first"]["counters"][k], (c["tag"], k, f)
        if c["first"]["model"] is None:
            assert r["counters"]["solutions"] == 0 and r["status"] == 0
        else:
            assert r["solutions"][0] == c["first"]["model"], (c["tag"], f)
        if "full" in c:
            r = oracle.dpll(f, "sound", max_solutions=0, sol_cap=1)
            for k in SOUND_CTR:
                assert r["counters"][k] == c["full"]["counters"][k], (c["tag"], k, f)
            assert r["counters"]["solutions"] == c["full"]["solutions"]
            assert (r["solutions"][0] if r["solutions"] else None) == c["full"]["first_solution"]


def test_cdcl_matches_reference_class(golden_dir):
    """oracle/cdcl_oracle.c against the reference's own CDCLSolver
    (tests/golden/cdcl_ref.json, make_golden_cdcl.py): verdict, the assignment
    dict in insertion order, decision level, var_inc (bit-exact float64), formula
    length, watch-list keys and the loop's counts -- also where the reference's
    unbounded loop was stopped after max_iter iterations."""
    cases = _load(golden_dir, "cdcl_ref.json")
    assert len(cases) >= 150 and {c["result"] for c in cases} >= {0, 1, -1}
    for c in cases:
        r = oracle.cdcl(c["formula"], c["max_iter"])
        assert r["result"] == c["result"], c["formula"]
        assert r["assignment"] == c["assignment"], c["formula"]
        assert r["var_inc"] == c["var_inc"]
        assert r["stats"]["level"] == c["level"]
        assert r["stats"]["clauses"] == c["clauses"] and r["stats"]["watch_keys"] == c["watch_keys"]
        for k in ("iterations", "conflicts", "decisions", "learned"):
            assert r["stats"][k] == c["stats"][k], (k, c["formula"])


def test_fullsolve_fixture_regenerates(golden_dir):
    """tests/golden/fullsolve_uf250.json (make_fullsolve.py): the instances
    regenerate bit-identically from their seed, and the oracle reproduces the
    recorded searches that finish quickly (the long ones are the GPU test's)."""
    import hashlib

    from satmi import cnf
    with open(os.path.join(golden_dir, "fullsolve_uf250.json")) as fh:
        g = json.load(fh)
    batch = cnf.uniform_ksat(g["count"], g["n"], g["m"], g["k"], seed=g["seed"])
    assert hashlib.sha256(batch.lits.tobytes()).hexdigest() == g["lits_sha256"]
    for c in g["cases"]:
        if c["counters"]["nodes"] > 20000:
            continue
        o = oracle.dpll(batch.instance(c["index"]), "sound", max_solutions=1, sol_cap=1)
        assert o["status"] == c["status"]
        assert o["counters"] == c["counters"]
        assert (o["solutions"][0] if o["solutions"] else []) == c["model"]
