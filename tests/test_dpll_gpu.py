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


# BASELINE configs[4]: uf250-1065-shaped 3-SAT and random 5-SAT n=200 at the
# 5-SAT threshold (alpha=21.117, m=4,223 -- the LDS-pressure layout: one wave
# per CU).  Full searches take 10^6+ calls for this heuristic, so parity is
# checked on node-capped searches: status, all counters and any model match the
# oracle bit-exactly at the cap.
@pytest.mark.parametrize("n,m,k,cap", [(250, 1065, 3, 1500), (200, 4223, 5, 600)])
def test_configs4_node_capped_parity(n, m, k, cap):
    B = 6
    batch = cnf.uniform_ksat(B, n, m, k, seed=4 * n + k)
    r = dpll_batch(batch, mode="sound", max_solutions=1, node_limit=cap, sol_cap=1)
    for b in range(B):
        o = oracle.dpll(batch.instance(b), "sound", max_solutions=1, node_limit=cap, sol_cap=1)
        assert int(r.status[b]) == o["status"], b
        got = r.counter_dict(b)
        for key in CTR:
            assert got[key] == o["counters"][key], (b, key)
        assert r.solutions(b)[:1] == o["solutions"][:1]


@pytest.mark.parametrize("n,m,k,cap,B", [(250, 1065, 3, 4000, 512), (200, 4223, 5, 1500, 256)])
def test_configs4_batch_properties(n, m, k, cap, B):
    batch = cnf.uniform_ksat(B, n, m, k, seed=n + 31 * k)
    r = dpll_batch(batch, mode="sound", max_solutions=1, node_limit=cap, sol_cap=1)
    ok = (_capi.DPLL_STOPPED, _capi.DPLL_EXHAUSTED, _capi.DPLL_NODE_LIMIT)
    for b in range(B):
        assert int(r.status[b]) in ok
        nodes = r.counter_dict(b)["nodes"]
        if r.status[b] == _capi.DPLL_NODE_LIMIT:
            assert nodes == cap + 1
        else:
            assert nodes <= cap
        if r.num_solutions(b):
            assert _satisfies(batch.instance(b), r.solutions(b)[0])
    # exact on a sample, at the batch's own cap
    for b in (0, B // 2, B - 1):
        o = oracle.dpll(batch.instance(b), "sound", max_solutions=1, node_limit=cap, sol_cap=1)
        assert int(r.status[b]) == o["status"]
        assert r.counter_dict(b) == {**r.counter_dict(b), **{k_: o["counters"][k_] for k_ in CTR}}


@pytest.mark.parametrize("fixture,min_unsat", [("uf250", 0), ("unsat150", 5), ("unsat200", 5), ("uuf250", 5),
                                               ("5sat200", 0)])
@pytest.mark.parametrize("split", [_capi.SPLIT_OFF, _capi.SPLIT_ALWAYS])
def test_configs4_solved_to_completion(golden_dir, fixture, min_unsat, split):
    """configs[4]-scale searches run to the end (no node cap): uf250-shaped SAT
    searches of 10^3-10^6 calls, UNSAT searches at n=150 / n=200, the
    uuf250 shape itself (n=250, m=1065: 6 UNSAT searches of 2.5-8.5 M calls
    that exhaust both branches of every decision, REF.py:167-214, beside 10
    SAT ones), and 64 random 5-SAT n=200 searches (m=2400: five 12-bit codes
    per clause word, the 5-literal LDS layout; 77 - 2.6e5 calls each) -- all
    decided: status, every counter and the model equal the oracle's
    (tests/golden/fullsolve_<fixture>.json, make_fullsolve.py), with and
    without branch splitting (a few searches on thousands of idle waves:
    helpers take subtrees of searches millions of calls deep).  Unsplit, a
    search runs on one wavefront, so only the searches of <= 2 M calls run."""
    with open(os.path.join(golden_dir, f"fullsolve_{fixture}.json")) as fh:
        g = json.load(fh)
    batch = cnf.uniform_ksat(g["count"], g["n"], g["m"], g["k"], seed=g["seed"])
    import hashlib
    assert hashlib.sha256(batch.lits.tobytes()).hexdigest() == g["lits_sha256"]
    cases = g["cases"]
    assert len(cases) >= 8
    assert sum(c["status"] == _capi.DPLL_EXHAUSTED for c in cases) >= min_unsat
    if split == _capi.SPLIT_OFF:
        cases = [c for c in cases if c["counters"]["nodes"] <= 2_000_000]
        assert cases
    fs = [batch.instance(c["index"]) for c in cases]   # only the searches the oracle finished
    _capi.set_split(split)
    try:
        r = dpll_batch(fs, mode="sound", max_solutions=1, sol_cap=1)   # a time limit would disable splitting
    finally:
        _capi.set_split(_capi.SPLIT_AUTO)
    for b, c in enumerate(cases):
        assert int(r.status[b]) == c["status"], c["index"]
        got = r.counter_dict(b)
        for key in CTR:
            assert got[key] == c["counters"][key], (c["index"], key)
        assert r.solutions(b)[:1] == ([c["model"]] if c["model"] else []), c["index"]
        if c["model"]:
            assert _satisfies(fs[b], c["model"])


def _random_mix(seed, count, nmax, kmax, mmax):
    rng = random.Random(seed)
    fs = []
    for _ in range(count):
        n = rng.randint(1, nmax)
        m = rng.randint(1, mmax)
        f = []
        for _ in range(m):
            k = rng.randint(1, min(kmax, n))
            f.append([v if rng.random() < 0.5 else -v for v in rng.sample(range(1, n + 1), k)])
        if rng.random() < 0.2 and f:   # duplicate literals and tautologies, as REF.py accepts them
            c = f[rng.randrange(len(f))]
            if len(c) < kmax:
                c.append(c[0] if rng.random() < 0.5 else -c[0])
        fs.append(f)
    return fs


def _run_policy(batch, policy, **kw):
    _capi.set_kernel(policy)
    try:
        return dpll_batch(batch, mode="sound", **kw)
    finally:
        _capi.set_kernel(_capi.KERNEL_AUTO)


@pytest.mark.parametrize("seed,nmax,kmax,mmax", [(1, 12, 3, 60), (2, 20, 5, 120), (3, 600, 3, 40)])
def test_scan_kernel_matches_general_and_oracle(seed, nmax, kmax, mmax):
    """The clause-scan kernel (dpll_scan.hip) against the general kernel and the
    oracle: SOUND mode, first model and full enumeration, every counter."""
    fs = _random_mix(seed, 240, nmax, kmax, mmax)
    for maxs, cap in ((1, 1), (0, 32)):
        rg = _run_policy(fs, _capi.KERNEL_GENERAL, max_solutions=maxs, sol_cap=cap, time_limit=20.0)
        for kern in (_capi.KERNEL_SCAN, _capi.KERNEL_INC):
            rs = _run_policy(fs, kern, max_solutions=maxs, sol_cap=cap, time_limit=20.0)
            assert (rs.status == rg.status).all()
            assert (rs.counters[:, :7] == rg.counters[:, :7]).all()
            assert (rs.root_len == rg.root_len).all()
            for b, f in enumerate(fs):
                assert rs.solutions(b) == rg.solutions(b), (kern, f)
                assert rs.root_assignment(b) == rg.root_assignment(b)
        for b in range(0, len(fs), 7):
            o = oracle.dpll(fs[b], "sound", max_solutions=maxs, sol_cap=cap)
            for key in CTR:
                assert rs.counter_dict(b)[key] == o["counters"][key], (key, fs[b])
            assert rs.solutions(b) == o["solutions"][:cap]


def test_scan_kernel_full_size_matches_general():
    batch = cnf.uniform_ksat(2048, 100, 426, 3, seed=77)
    rg = _run_policy(batch, _capi.KERNEL_GENERAL, max_solutions=1, sol_cap=1)
    for kern in (_capi.KERNEL_SCAN, _capi.KERNEL_INC):
        rs = _run_policy(batch, kern, max_solutions=1, sol_cap=1)
        assert (rs.status == rg.status).all()
        assert (rs.counters[:, :7] == rg.counters[:, :7]).all()
        assert (rs.sol_lits == rg.sol_lits).all()


def _mass_unit_formulas(seed, count):
    """16-bit-code formulas (n > 127) whose snapshots exceed the 512 entries the
    scan kernel keeps in LDS (the rest go to the wave's HBM scratch): a hub
    variable in 520-900 binary clauses [-1, l] (its True branch makes them all
    unit at once) or 520-700 unit clauses at the root, plus random 3-clauses.
    The unit literals repeat (a variable's first occurrence wins, some first
    occurrences lie past entry 512) with one sign per variable (the whole
    snapshot is assigned: every clause holds a literal of that sign) or with
    random signs (a conflict cuts it)."""
    rng = random.Random(seed)
    fs = []
    for i in range(count):
        n = rng.randint(130, 250)
        sign = [1 if rng.random() < 0.5 else -1 for _ in range(n + 1)]
        lit = lambda: rng.randint(2, n) * (1 if rng.random() < 0.5 else -1)   # noqa: E731
        ulit = (lambda: (lambda v: v * sign[v])(rng.randint(2, n))) if i % 2 == 0 else lit   # noqa: E731
        if i % 3 == 2:
            f = [[ulit()] for _ in range(rng.randint(520, 700))]
        else:   # the hub occurs both ways (not pure), and most in the binary clauses: branched on first
            f = [[-1, ulit()] for _ in range(rng.randint(520, 900))] + [[1, lit(), lit()] for _ in range(20)]
        f += [[ulit(), lit(), lit()] for _ in range(rng.randint(n // 2, n))]
        rng.shuffle(f)
        fs.append(f)
    return fs


def test_snapshot_past_lds_entries_matches_general_and_oracle():
    fs = _mass_unit_formulas(91, 36)
    rg = _run_policy(fs, _capi.KERNEL_GENERAL, max_solutions=1, sol_cap=1, node_limit=3000)
    for kern in (_capi.KERNEL_SCAN, _capi.KERNEL_INC):
        rs = _run_policy(fs, kern, max_solutions=1, sol_cap=1, node_limit=3000)
        assert (rs.status == rg.status).all(), kern
        assert (rs.counters[:, :7] == rg.counters[:, :7]).all(), kern
        for b in range(len(fs)):
            assert rs.solutions(b) == rg.solutions(b), (kern, b)
    assert (rg.counters[:, 2] > 0).all()   # unit propagations happened in every instance
    for b in range(0, len(fs), 3):
        o = oracle.dpll(fs[b], "sound", max_solutions=1, sol_cap=1, node_limit=3000)
        for key in CTR:
            assert rs.counter_dict(b)[key] == o["counters"][key], (key, b)
        assert rs.solutions(b) == o["solutions"][:1]


def test_scan_policy_rejects_ineligible():
    f = [[1, 2], [-1, 2], []]
    for kern in (_capi.KERNEL_SCAN, _capi.KERNEL_INC):
        _capi.set_kernel(kern)
        try:
            with pytest.raises(_capi.SatmiError):
                dpll_batch([f], mode="sound", max_solutions=1)      # an empty clause
            with pytest.raises(_capi.SatmiError):
                dpll_batch([[[1, 2]]], mode="ref", max_solutions=0)  # REF mode
        finally:
            _capi.set_kernel(_capi.KERNEL_AUTO)


def test_scan_broken_length_promise_is_too_large():
    import torch
    # 5-literal clauses under a promise of <= 3 (the 3-slot clause packing)
    batch = cnf.uniform_ksat(4, 20, 60, 5, seed=5)
    dev = torch.device("cuda", 0)
    t = [torch.from_numpy(a).to(dev) for a in (batch.inst_clause_begin, batch.clause_lit_begin, batch.lits,
                                             batch.inst_nvars)]
    st = torch.zeros(4, dtype=torch.int32, device=dev)
    ctr = torch.zeros((4, 8), dtype=torch.int64, device=dev)
    sl = torch.zeros(4, dtype=torch.int32, device=dev)
    so = torch.zeros((4, 20), dtype=torch.int32, device=dev)
    L = _capi.load()
    rc = L.satmi_dpll_batch_device(4, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), 20, 60,
                                   300, 3, None, None, _capi.MODE_SOUND, 1, 0, 0.0, 1, 20, st.data_ptr(),
                                   ctr.data_ptr(), sl.data_ptr(), so.data_ptr(), None, None, None)
    _capi.check(rc, "satmi_dpll_batch_device")
    torch.cuda.synchronize()
    assert (st.cpu() == _capi.DPLL_TOO_LARGE).all()


def test_concurrent_streams_keep_separate_work_queues():
    """Two batches launched on two streams at once (bench.py's pipelined steps)
    each draw from their own stream's work counter: results equal the
    one-at-a-time host path."""
    import torch

    dev = torch.device("cuda", 0)
    L = _capi.load()
    n, m, k, B = 60, 256, 3, 2048
    runs = []
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    for j, s in enumerate(streams):
        icb, clb, lits, nv = cnf.uniform_ksat_device(B, n, m, k, seed=77 + j, device=dev)
        out = (torch.zeros(B, dtype=torch.int32, device=dev),
               torch.zeros((B, _capi.NCOUNTERS), dtype=torch.int64, device=dev),
               torch.zeros(B, dtype=torch.int32, device=dev),
               torch.zeros((B, n), dtype=torch.int32, device=dev))
        runs.append(((icb, clb, lits, nv), out))
    torch.cuda.synchronize()
    for (batch, out), s in zip(runs, streams):
        icb, clb, lits, nv = batch
        st, ctr, sl, sol = out
        rc = L.satmi_dpll_batch_device(B, icb.data_ptr(), clb.data_ptr(), lits.data_ptr(), nv.data_ptr(), n, m,
                                       m * k, k, None, None, _capi.MODE_SOUND, 1, 0, 0.0, 1, n, st.data_ptr(),
                                       ctr.data_ptr(), sl.data_ptr(), sol.data_ptr(), None, None, s.cuda_stream)
        _capi.check(rc, "satmi_dpll_batch_device")
    torch.cuda.synchronize()
    for (batch, out) in runs:
        host = cnf.CnfBatch(*(t.cpu().numpy() for t in batch))
        ref = dpll_batch(host, mode="sound", max_solutions=1)
        st, ctr, sl, sol = (t.cpu().numpy() for t in out)
        assert (st == ref.status).all()
        assert (ctr[:, :7] == ref.counters[:, :7]).all()
        assert (sl == ref.sol_len[:, 0]).all()


def test_snapshot_epoch_wraparound_parity():
    """The scan kernel tags unit-snapshot stamps with a 16-bit epoch (one per
    snapshot) and resets every stamp when the epoch nears its limit
    (dpll_scan.hip, next_decision_epoch).  A uf250-shaped search of 20,000
    calls uses > 65,536 epochs, so the reset runs, and every counter and the
    model must still equal the oracle's."""
    n, m, k, cap = 250, 1065, 3, 20000
    batch = cnf.uniform_ksat(2, n, m, k, seed=2026)
    r = dpll_batch(batch, mode="sound", max_solutions=1, node_limit=cap, sol_cap=1)
    epochs = [int(r.counters[b, 6] + r.counters[b, 1]) for b in range(2)]   # rounds + decisions
    assert max(epochs) > 65536, epochs
    for b in range(2):
        o = oracle.dpll(batch.instance(b), "sound", max_solutions=1, node_limit=cap, sol_cap=1)
        assert int(r.status[b]) == o["status"], b
        got = r.counter_dict(b)
        for key in CTR:
            assert got[key] == o["counters"][key], (b, key)
        assert r.solutions(b)[:1] == o["solutions"][:1]


@pytest.mark.parametrize("policy", ["scan", "inc", "general"])
def test_sound_kernels_match_reference_fixture(golden_dir, policy):
    """Both DPLL kernels against tests/golden/dpll_sound_ref.json: the reference's
    own dpll_optimized with only the branch of REF.py:210-213 applied as a unit
    clause (make_golden_sound.py), at BASELINE configs[1] (n=50) and configs[2]
    (n=100) shapes plus edge and generator formulas.  First-model search (the
    bench's max_solutions=1): every counter and the model; full enumeration:
    every counter and the solution count."""
    cases = _golden(golden_dir, "dpll_sound_ref.json")
    kern = {"scan": _capi.KERNEL_SCAN, "inc": _capi.KERNEL_INC, "general": _capi.KERNEL_GENERAL}[policy]
    if policy != "general":   # the clause kernels' shapes: clauses of 1..5 literals
        cases = [c for c in cases if c["formula"] and all(1 <= len(cl) <= 5 for cl in c["formula"])]
    assert sum(c["tag"] == "configs2_n100" for c in cases) >= 48
    fs = [c["formula"] for c in cases]
    r = _run_policy(fs, kern, max_solutions=1, sol_cap=1, time_limit=60.0)
    for b, c in enumerate(cases):
        got = r.counter_dict(b)
        for k in ("nodes", "decisions", "unit_props", "pure_assigns", "conflicts"):
            assert got[k] == c["first"]["counters"][k], (policy, c["tag"], k)
        want = [] if c["first"]["model"] is None else [c["first"]["model"]]
        assert r.solutions(b) == want, (policy, c["tag"])
    full = [c for c in cases if "full" in c]
    r = _run_policy([c["formula"] for c in full], kern, max_solutions=0, sol_cap=1, time_limit=60.0)
    for b, c in enumerate(full):
        assert int(r.status[b]) == _capi.DPLL_EXHAUSTED
        got = r.counter_dict(b)
        for k in ("nodes", "decisions", "unit_props", "pure_assigns", "conflicts"):
            assert got[k] == c["full"]["counters"][k], (policy, c["tag"], k)
        assert got["solutions"] == c["full"]["solutions"]
        first = r.solutions(b)[0] if got["solutions"] else None
        assert first == c["full"]["first_solution"], (policy, c["tag"])


@pytest.mark.parametrize("tag", ["configs1_n50", "configs2_n100"])
@pytest.mark.parametrize("split", [_capi.SPLIT_OFF, _capi.SPLIT_ALWAYS])
def test_bench_kernel_matches_reference_fixture(golden_dir, tag, split):
    """The kernel behind the headline (dpll_fixed_kernel: K = 3, n <= 127,
    m <= 448) directly against the reference's own vectors of the bench
    shapes (tests/golden/dpll_sound_ref.json, make_golden_sound.py), one K = 3
    batch per tag so that the launch takes the fixed class; unsplit, and split
    with every search allowed to donate from its first check (warm-up 0)."""
    cases = [c for c in _golden(golden_dir, "dpll_sound_ref.json") if c["tag"] == tag]
    assert len(cases) >= 64
    fs = [c["formula"] for c in cases]
    n = max(abs(l) for f in fs for cl in f for l in cl)
    m = max(len(f) for f in fs)
    assert all(len(cl) == 3 for f in fs for cl in f)
    kern, lds, _ = _capi.plan(n, m, 3 * m, 3)
    assert kern == _capi.KERNEL_INC and lds == 5108, "not dpll_fixed_kernel's shape class"
    _capi.set_split(split)
    _capi.set_split_warmup(0)
    try:
        r = dpll_batch(fs, mode="sound", max_solutions=1, sol_cap=1)
    finally:
        _capi.set_split(True)
        _capi.set_split_warmup(-1)
    for b, c in enumerate(cases):
        got = r.counter_dict(b)
        for k in ("nodes", "decisions", "unit_props", "pure_assigns", "conflicts"):
            assert got[k] == c["first"]["counters"][k], (tag, b, k)
        want = [] if c["first"]["model"] is None else [c["first"]["model"]]
        assert r.solutions(b) == want, (tag, b)


@pytest.mark.parametrize("n,m,cap", [(200, 700, 800), (300, 1100, 500), (500, 2130, 400), (480, 2400, 400)])
def test_scan_kernel_chunk_group_tails(n, m, cap):
    """Clause counts whose 64-clause chunks split into a 7-chunk group followed
    by a 4-chunk group (m=700: 11 chunks; m=1100: 7+7+4 = 18 chunks) -- the
    for_chunks path of dpll_scan.hip no other shape reaches -- and 3-SAT with
    more than 2,048 clauses (m=2130, 2400: unit bitmaps of 67 / 75 words, the
    multi-word placement loop of the one-step unit scan's bitmap path, ADVICE
    r04).  Scan kernel vs general kernel vs oracle, node-capped, every counter
    and any model."""
    batch = cnf.uniform_ksat(6, n, m, 3, seed=n + m)
    rg = _run_policy(batch, _capi.KERNEL_GENERAL, max_solutions=1, node_limit=cap, sol_cap=1)
    ri = _run_policy(batch, _capi.KERNEL_INC, max_solutions=1, node_limit=cap, sol_cap=1)
    rs = _run_policy(batch, _capi.KERNEL_SCAN, max_solutions=1, node_limit=cap, sol_cap=1)
    for r in (rs, ri):
        assert (r.status == rg.status).all()
        assert (r.counters[:, :7] == rg.counters[:, :7]).all()
    for b in range(6):
        o = oracle.dpll(batch.instance(b), "sound", max_solutions=1, node_limit=cap, sol_cap=1)
        assert int(rs.status[b]) == o["status"]
        for key in CTR:
            assert rs.counter_dict(b)[key] == o["counters"][key], (b, key)
        assert rs.solutions(b)[:1] == o["solutions"][:1]


def _run_split(batch, split, policy=_capi.KERNEL_AUTO, warmup=0, **kw):
    # warm-up 0: every search may donate from its first check (the protocol
    # under the most stress; the default only splits long searches)
    _capi.set_split(_capi.SPLIT_ALWAYS if split else _capi.SPLIT_OFF)
    _capi.set_split_warmup(warmup)
    try:
        return _run_policy(batch, policy, **kw)
    finally:
        _capi.set_split(True)
        _capi.set_split_warmup(-1)


@pytest.mark.parametrize("n,m,B,policy", [(100, 426, 24, _capi.KERNEL_AUTO), (100, 426, 3000, _capi.KERNEL_AUTO),
                                          (50, 213, 40, _capi.KERNEL_AUTO), (140, 596, 16, _capi.KERNEL_INC),
                                          (100, 426, 24, _capi.KERNEL_SCAN)])
def test_branch_splitting_matches_unsplit(n, m, B, policy):
    """Branch splitting (dpll_scan.hip, "Splitting the tail"): a batch far
    smaller than the resident waves makes nearly every search donate subtrees
    to idle waves (and helpers donate further); statuses, every counter and
    the models must equal the unsplit search, and the oracle on a sample."""
    batch = cnf.uniform_ksat(B, n, m, 3, seed=n * B + m)
    ru = _run_split(batch, False, policy, max_solutions=1, sol_cap=1)
    rs = _run_split(batch, True, policy, max_solutions=1, sol_cap=1)
    assert (rs.status == ru.status).all()
    assert (rs.counters[:, :7] == ru.counters[:, :7]).all()
    assert (rs.sol_len == ru.sol_len).all()
    assert (rs.sol_lits == ru.sol_lits).all()
    for b in range(0, B, max(1, B // 6)):
        o = oracle.dpll(batch.instance(b), "sound", max_solutions=1, sol_cap=1)
        for key in CTR:
            assert rs.counter_dict(b)[key] == o["counters"][key], (b, key)
        assert rs.solutions(b)[:1] == o["solutions"][:1]


def test_branch_splitting_repeated_launches_one_stream():
    """Slot states are tagged per launch (the pool is never cleared): many
    back-to-back split launches on one stream stay exact."""
    batch = cnf.uniform_ksat(32, 100, 426, 3, seed=99)
    ru = _run_split(batch, False, max_solutions=1, sol_cap=1)
    for _ in range(6):
        rs = _run_split(batch, True, max_solutions=1, sol_cap=1)
        assert (rs.counters[:, :7] == ru.counters[:, :7]).all()
        assert (rs.sol_lits == ru.sol_lits).all()


def test_split_stats_reset_by_a_launch_that_does_not_split():
    """satmi_dpll_split_stats reports the stream's LAST launch: after a split
    launch, a launch of the general kernel (REF mode) on the same stream
    leaves the statistics all zero (include/satmi.h contract)."""
    batch = cnf.uniform_ksat(32, 100, 426, 3, seed=99)
    _run_split(batch, True, max_solutions=1, sol_cap=1)
    st = _capi.split_stats(None)
    assert st["done"] > 0 and st["donations"] > 0
    dpll_batch([[[1, 2], [-1, 2], [1, -2]]], mode="ref", max_solutions=0, sol_cap=8)   # dpll_batch_kernel
    assert all(v == 0 for v in _capi.split_stats(None).values())
    _run_split(batch, True, max_solutions=1, sol_cap=1)
    assert _capi.split_stats(None)["done"] > 0
    _capi.set_kernel(_capi.KERNEL_WIDE)
    try:
        dpll_batch([[[1, 2], [-1, 2], [1, -2]]], mode="ref", max_solutions=0, sol_cap=8)   # dpll_wide_kernel
    finally:
        _capi.set_kernel(_capi.KERNEL_AUTO)
    assert all(v == 0 for v in _capi.split_stats(None).values())


@pytest.mark.parametrize("seed,nmax,kmax,mmax", [(11, 12, 4, 60), (12, 400, 300, 30)])
def test_wide_kernel_matches_general_and_oracle(seed, nmax, kmax, mmax):
    """The general kernel's wide form (per-wave HBM arena, 32-bit indices,
    SATMI_KERNEL_WIDE) against its LDS form and the oracle, REF and SOUND
    modes, first model and full enumeration: every counter, every solution,
    the root assignment.  kmax=300 reaches clauses past the LDS form's
    255-literal limit (there only the oracle is the reference)."""
    fs = _random_mix(seed, 160, nmax, kmax, mmax)
    long_clause = any(len(c) > 255 for f in fs for c in f)
    for mode, maxs, cap in (("ref", 0, 32), ("sound", 1, 1), ("sound", 0, 32)):
        _capi.set_kernel(_capi.KERNEL_WIDE)
        try:
            rw = dpll_batch(fs, mode=mode, max_solutions=maxs, sol_cap=cap, node_limit=3000)
        finally:
            _capi.set_kernel(_capi.KERNEL_AUTO)
        if not long_clause:
            _capi.set_kernel(_capi.KERNEL_GENERAL)
            try:
                rg = dpll_batch(fs, mode=mode, max_solutions=maxs, sol_cap=cap, node_limit=3000)
            finally:
                _capi.set_kernel(_capi.KERNEL_AUTO)
            assert (rw.status == rg.status).all()
            assert (rw.counters[:, :7] == rg.counters[:, :7]).all()
            assert (rw.root_len == rg.root_len).all()
        for b in range(0, len(fs), 1 if long_clause else 5):
            o = oracle.dpll(fs[b], mode, max_solutions=maxs, node_limit=3000, sol_cap=cap)
            assert int(rw.status[b]) == o["status"], (mode, b)
            for key in CTR:
                assert rw.counter_dict(b)[key] == o["counters"][key], (mode, key, b)
            assert rw.solutions(b) == o["solutions"][:cap], (mode, b)
            assert rw.root_assignment(b) == o["root_assign"]


def test_wide_kernel_reference_golden(golden_dir):
    cases = _golden(golden_dir, "dpll_ref.json")
    cap = max(len(c["solutions"]) for c in cases) + 1
    _capi.set_kernel(_capi.KERNEL_WIDE)
    try:
        r = dpll_batch([c["formula"] for c in cases], mode="ref", max_solutions=0, sol_cap=cap,
                       inits=[c["init"] for c in cases], time_limit=20.0)
    finally:
        _capi.set_kernel(_capi.KERNEL_AUTO)
    for b, c in enumerate(cases):
        assert r.solutions(b) == c["solutions"]
        got = r.counter_dict(b)
        for k, v in c["counters"].items():
            assert got[k] == v, (k, c["formula"])


@pytest.mark.parametrize("clauses,max_len,nvars,cap", [(1000, 100, 100, 40), (5000, 1000, 1000, 4)])
def test_reference_menu_shapes_run_wide(clauses, max_len, nvars, cap):
    """The reference's own menu runs beyond one wave's LDS image: rezultat.txt:248-250
    (1000 clauses, avg length ~50, 100 variables) and :488-490 (5000 clauses, avg
    length ~500, 1000 variables), drawn with REF.py:21-29's generator.  AUTO
    dispatch takes the wide kernel; node-capped REF and SOUND searches equal the
    oracle (status, counters, solutions)."""
    from satmi.solvers import generate_large_formula
    random.seed(clauses + nvars)
    f = generate_large_formula(clauses, max_len, nvars)
    L = sum(len(c) for c in f)
    kern, _, _ = _capi.plan(nvars, clauses, L, max(len(c) for c in f), mode=_capi.MODE_REF)
    assert kern == _capi.KERNEL_WIDE
    for mode, maxs in (("ref", 0), ("sound", 1)):
        r = dpll_batch([f], mode=mode, max_solutions=maxs, node_limit=cap, sol_cap=4)
        o = oracle.dpll(f, mode, max_solutions=maxs, node_limit=cap, sol_cap=4)
        assert int(r.status[0]) == o["status"]
        for key in CTR:
            assert r.counter_dict(0)[key] == o["counters"][key], (mode, key)
        assert r.solutions(0) == o["solutions"][:4]
        assert r.root_assignment(0) == o["root_assign"]
