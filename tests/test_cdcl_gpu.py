"""GPU parity of the CDCL kernel (csrc/cdcl.hip) through the C ABI: against the
reference's own CDCLSolver (tests/golden/cdcl_ref.json) and the oracle
(oracle/cdcl_oracle.c) -- verdict, the assignment dict in insertion order,
var_inc bit for bit, decision level and the loop's counts."""
import json
import os
import random

import pytest

import oracle
from satmi.cdcl import CDCL_SAT, CDCL_UNSAT, CDCL_LIMIT, cdcl_batch

pytestmark = pytest.mark.gpu

STATUS = {1: CDCL_SAT, 0: CDCL_UNSAT, -1: CDCL_LIMIT}


def _check(r, want_result, want_assign, want_var_inc, want_stats):
    assert r["status"] == STATUS[want_result]
    assert r["assignment"] == want_assign
    assert r["var_inc"] == want_var_inc
    for k, v in want_stats.items():
        assert r["stats"][k] == v, k


def test_cdcl_matches_reference_class(golden_dir):
    with open(os.path.join(golden_dir, "cdcl_ref.json")) as fh:
        cases = json.load(fh)["cases"]
    by_cap = {}
    for c in cases:
        by_cap.setdefault(c["max_iter"], []).append(c)
    for cap, cs in by_cap.items():
        rs = cdcl_batch([c["formula"] for c in cs], max_iter=cap)
        for r, c in zip(rs, cs):
            want = {k: c["stats"][k] for k in ("iterations", "conflicts", "decisions", "learned")}
            want.update(level=c["level"], clauses=c["clauses"], watch_keys=c["watch_keys"])
            _check(r, c["result"], c["assignment"], c["var_inc"], want)


@pytest.mark.parametrize("seed,count,nmax,kmax,cap", [(1, 200, 16, 4, 3000), (2, 64, 40, 6, 20000)])
def test_cdcl_matches_oracle_random(seed, count, nmax, kmax, cap):
    """Random formulas (repeated literals and tautologies included) on long
    runs: the set tables resize, dummies recycle, var_inc drifts."""
    rng = random.Random(seed)
    fs = []
    for _ in range(count):
        n = rng.randint(2, nmax)
        f = []
        for _ in range(rng.randint(1, 5 * n)):
            k = rng.randint(1, min(kmax, n))
            c = [v if rng.random() < 0.5 else -v for v in rng.sample(range(1, n + 1), k)]
            if rng.random() < 0.1:
                c.append(c[0] if rng.random() < 0.5 else -c[0])
            f.append(c)
        fs.append(f)
    rs = cdcl_batch(fs, max_iter=cap)
    for f, r in zip(fs, rs):
        o = oracle.cdcl(f, cap)
        _check(r, o["result"], o["assignment"], o["var_inc"],
               {k: o["stats"][k] for k in ("iterations", "conflicts", "decisions", "learned", "clauses",
                                           "watch_keys", "level")})


def test_cdcl_drop_in_and_driver_row():
    from satmi import driver
    from satmi.solvers import cdcl_solve
    f = [[1, 2], [-1, 2], [-2, 3]]
    o = oracle.cdcl(f)
    sat, model = cdcl_solve([list(c) for c in f])
    assert sat and list(model.items()) == [(abs(l), l > 0) for l in o["assignment"]]
    # [[-1, -2]] loops forever in the reference (rezultat.txt's CDCL timeouts): a timeout row
    results = driver.run_solvers([[-1, -2]], [("CDCL", cdcl_solve)], timeout=1, print_fn=lambda *a: None)
    assert results["CDCL"]["output"] == "Timeout after 1 seconds"


def test_cdcl_long_clauses_of_repeated_literals():
    """Clauses repeating their literals many times (the reference accepts them):
    conflict clauses longer than 2 x variables + 2 entries, the learned-literal
    lists' old bound (csrc/cdcl.hip analyze_conflict), against the oracle."""
    rng = random.Random(11)
    fs = []
    for _ in range(120):
        n = rng.randint(2, 5)
        f = []
        for _ in range(rng.randint(2, 4 * n)):
            c = [v if rng.random() < 0.5 else -v for v in rng.sample(range(1, n + 1), rng.randint(1, n))]
            c = c * rng.randint(2, 6)   # every literal repeated: up to 6n entries
            rng.shuffle(c)
            f.append(c)
        fs.append(f)
    rs = cdcl_batch(fs, max_iter=2000)
    for f, r in zip(fs, rs):
        o = oracle.cdcl(f, 2000)
        _check(r, o["result"], o["assignment"], o["var_inc"],
               {k: o["stats"][k] for k in ("iterations", "conflicts", "decisions", "learned", "clauses",
                                           "watch_keys", "level")})


def test_cdcl_concurrent_calls_from_threads():
    """satmi_cdcl_batch_host from several host threads at once (one arena and
    stream per concurrent call): every call's outputs equal the same batch run
    alone, in both return forms."""
    from concurrent.futures import ThreadPoolExecutor

    from satmi import cnf
    from satmi.cdcl import cdcl_batch_packed
    batches = [cnf.menu_batch(512, 80, 3, 15, seed=900 + t) for t in range(6)]
    alone = [cdcl_batch_packed(b, max_iter=3000, arrays=True) for b in batches]
    with ThreadPoolExecutor(6) as ex:
        for _ in range(2):
            together = list(ex.map(lambda b: cdcl_batch_packed(b, max_iter=3000, arrays=True), batches))
            for a, t in zip(alone, together):
                for key in ("status", "assign_len", "stats", "var_inc"):
                    assert (a[key] == t[key]).all(), key
                for i in range(len(a["status"])):   # models: the first assign_len entries of a row
                    n = a["assign_len"][i]
                    assert (a["assign"][i, :n] == t["assign"][i, :n]).all(), i
    dicts = cdcl_batch_packed(batches[0], max_iter=3000)
    a = alone[0]
    for i in (0, 7, 511):
        assert dicts[i]["status"] == a["status"][i]
        assert dicts[i]["assignment"] == a["assign"][i, :a["assign_len"][i]].tolist()


def test_cdcl_arena_form_beyond_lds():
    """Formulas whose per-variable / per-key arrays exceed the LDS budget
    (csrc/cdcl.hip CDCL_LDS_MAX: ~85 B per variable, so > ~380 variables) run
    with those arrays in the HBM arena; a batch mixing them with small formulas
    (the launch takes the arena form for all) equals the oracle."""
    rng = random.Random(5)
    fs = []
    for n in (420, 600, 12, 9):
        f = []
        for _ in range(int(2.0 * n)):
            c = [v if rng.random() < 0.5 else -v for v in rng.sample(range(1, n + 1), 3)]
            f.append(c)
        fs.append(f)
    rs = cdcl_batch(fs, max_iter=400)
    for f, r in zip(fs, rs):
        o = oracle.cdcl(f, 400)
        _check(r, o["result"], o["assignment"], o["var_inc"],
               {k: o["stats"][k] for k in ("iterations", "conflicts", "decisions", "learned", "clauses",
                                           "watch_keys", "level")})


def test_cdcl_large_watch_tables():
    """Thousands of clauses watched by the same few literals: set tables grow
    past the register occupancy bitmap of a resize (csrc/cdcl.hip
    WS_BITMAP_SLOTS = 4,096 slots: beyond it the re-insertion probes memory),
    collide along linear-probe runs and perturbation, and fill with dummies as
    the watches move; against the oracle."""
    rng = random.Random(23)
    fs = []
    for n, m in ((10, 1500), (12, 2600), (8, 900), (14, 3200)):
        f = []
        for _ in range(m):
            first = rng.choice((1, -1, 2))   # few watch lists take most clauses
            rest = [v if rng.random() < 0.5 else -v for v in rng.sample(range(3, n + 1), rng.randint(1, 3))]
            f.append([first] + rest)
        fs.append(f)
    rs = cdcl_batch(fs, max_iter=300)
    for f, r in zip(fs, rs):
        o = oracle.cdcl(f, 300)
        _check(r, o["result"], o["assignment"], o["var_inc"],
               {k: o["stats"][k] for k in ("iterations", "conflicts", "decisions", "learned", "clauses",
                                           "watch_keys", "level")})
