"""Fixtures for configs[4] solved to completion (no node cap), SOUND mode,
first model:
    uf250      uf250-shaped random 3-SAT (n=250, m=1065): the searches that
               finish (all of them SAT) -- ~30 min on 8 cores
    unsat150   random 3-SAT n=150, m=639 (alpha 4.26): mostly UNSAT, searches
               exhausting both branches of every decision (~40 k nodes)
    unsat200   random 3-SAT n=200, m=852: UNSAT searches of 10^5-10^6 nodes
               (~1 min on 6 cores)
    uuf250     uuf250-shaped random 3-SAT (n=250, m=1065), node cap 5e7: the
               UNSAT searches at n=250 that exhaust both branches of every
               decision to the end (~1 h on 5 cores)
    5sat200    random 5-SAT n=200, m=2400 (alpha 12): configs[4]'s 5-SAT
               batches decided to the end.  At the 5-SAT threshold (alpha
               21.117, the node-capped bench leg) no search of 64 finished in
               90 s on the GPU, nor at alpha 17-19 in 30 s (tools/fullsolve_probe.py,
               profiles/r06/fullsolve_5sat_probe.txt); at alpha 12 all 64 finish
               (77 .. 2.6e5 nodes), which the oracle can follow
    python tests/golden/make_fullsolve.py [set]      (default: uf250)

The checker is the C oracle (oracle/sat_oracle.c, SOUND mode), itself pinned to
the reference's dpll_optimized with only its branch statement rewritten
(tests/golden/dpll_sound_ref.json, make_golden_sound.py) -- at n=250 the
reference's own Python would need hours per instance, so these vectors are the
oracle's.  Instances are regenerated from (seed, n, m, k) by
satmi.cnf.uniform_ksat; the sha256 of the literal array guards that.  An
instance the oracle does not finish within NODE_CAP nodes is dropped.
"""
import hashlib
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "sat-mpi-stana-andrei_amd"))
sys.path.insert(0, ROOT)

from satmi import cnf  # noqa: E402
from oracle import oracle  # noqa: E402

# set: (n, m, k, seed, count, node cap) -- the fixture keeps the searches that finish within the cap
SETS = {"uf250": (250, 1065, 3, 250, 96, 1_200_000),
        "unsat150": (150, 639, 3, 150, 24, 2_000_000),
        "unsat200": (200, 852, 3, 200, 12, 2_000_000),
        "uuf250": (250, 1065, 3, 2501, 16, 50_000_000),
        "5sat200": (200, 2400, 5, 5200, 64, 2_000_000)}
SET = sys.argv[1] if len(sys.argv) > 1 else "uf250"
N, M, K, SEED, COUNT, NODE_CAP = SETS[SET]
OUT = os.path.join(HERE, f"fullsolve_{SET}.json")


def solve(i):
    b = cnf.uniform_ksat(COUNT, N, M, K, seed=SEED)
    o = oracle.dpll(b.instance(i), "sound", max_solutions=1, node_limit=NODE_CAP, sol_cap=1)
    return i, o


def main():
    b = cnf.uniform_ksat(COUNT, N, M, K, seed=SEED)
    sha = hashlib.sha256(b.lits.tobytes()).hexdigest()
    cases = []
    with ProcessPoolExecutor(max_workers=int(os.environ.get("FULLSOLVE_WORKERS", min(6, os.cpu_count() or 1)))) as ex:
        for i, o in ex.map(solve, range(COUNT)):
            print(i, o["status"], o["counters"]["nodes"], flush=True)
            if o["counters"]["nodes"] > NODE_CAP:
                continue
            cases.append({"index": i, "status": o["status"], "counters": o["counters"],
                          "model": o["solutions"][0] if o["solutions"] else []})
    with open(OUT, "w") as fh:
        json.dump({"source": "oracle/sat_oracle.c SOUND mode via tests/golden/make_fullsolve.py",
                   "n": N, "m": M, "k": K, "seed": SEED, "count": COUNT, "lits_sha256": sha,
                   "node_cap": NODE_CAP, "cases": cases}, fh, separators=(",", ":"))
    print(f"{len(cases)} of {COUNT} solved -> {OUT}")


if __name__ == "__main__":
    main()
