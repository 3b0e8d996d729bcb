"""Fixtures for configs[4] solved to completion (no node cap): uf250-shaped
random 3-SAT (n=250, m=1065), SOUND mode, first model.

Run here (CPU, ~30 min on 8 cores):
    python tests/golden/make_fullsolve.py

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

N, M, K, SEED, COUNT = 250, 1065, 3, 250, 96
NODE_CAP = 1_200_000   # most uf250-shaped searches need more: the fixture keeps the ones that finish
OUT = os.path.join(HERE, "fullsolve_uf250.json")


def solve(i):
    b = cnf.uniform_ksat(COUNT, N, M, K, seed=SEED)
    o = oracle.dpll(b.instance(i), "sound", max_solutions=1, node_limit=NODE_CAP, sol_cap=1)
    return i, o


def main():
    b = cnf.uniform_ksat(COUNT, N, M, K, seed=SEED)
    sha = hashlib.sha256(b.lits.tobytes()).hexdigest()
    cases = []
    with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
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
