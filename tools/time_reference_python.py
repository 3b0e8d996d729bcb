"""Time the REFERENCE's own Python DPLL (SOUND rewrite of REF.py:210-213, as in
tests/golden/make_golden_sound.py) beside the C oracle on the same bench-shaped
instances, on one core of THIS container (the reference is not on the GPU box,
so bench.py's cpu_baseline is the C oracle; this gives the ratio between them).

    python tools/time_reference_python.py [--n 100] [--count 24] [--seconds 120]

UNSAT instances only: for them the first-model search is the whole search, so
the unmodified enumeration (no tracer, no early stop) times exactly the bench's
work.  Prints per-instance seconds and nodes/s for both, as one JSON line.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "sat-mpi-stana-andrei_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.setrecursionlimit(100000)

from satmi import cnf  # noqa: E402
from oracle import oracle  # noqa: E402
import make_golden_sound as ref  # noqa: E402  (loads the reference's functions, SOUND rewrite)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--count", type=int, default=24)
    ap.add_argument("--seconds", type=float, default=120.0)
    a = ap.parse_args()
    m = int(round(4.26 * a.n))
    batch = cnf.uniform_ksat(4 * a.count, a.n, m, 3, seed=4242)
    dpll = ref.NS["dpll_optimized"]
    py_t = c_t = 0.0
    nodes = 0
    done = 0
    for i in range(batch.num_instances):
        f = batch.instance(i)
        t = time.perf_counter()
        o = oracle.dpll(f, "sound", max_solutions=1, sol_cap=1)
        ct = time.perf_counter() - t
        if o["status"] != 0:          # keep UNSAT searches (first model = whole search)
            continue
        t = time.perf_counter()
        sols = dpll([list(c) for c in f], {})
        pt = time.perf_counter() - t
        assert sols == []
        py_t += pt
        c_t += ct
        nodes += o["counters"]["nodes"]
        done += 1
        if done >= a.count or py_t > a.seconds:
            break
    print(json.dumps({"n": a.n, "m": m, "unsat_instances": done, "nodes": nodes,
                      "reference_python_s_per_instance": py_t / done, "reference_python_nodes_per_s": nodes / py_t,
                      "c_oracle_s_per_instance": c_t / done, "c_oracle_nodes_per_s": nodes / c_t,
                      "python_over_c": py_t / c_t}))


if __name__ == "__main__":
    main()
