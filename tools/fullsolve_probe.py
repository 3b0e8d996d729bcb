"""How long do searches solved to the end take?  One batch of uniform random
k-SAT on the GPU (SOUND mode, first model, no node cap, branch splitting
always), each search bounded by a time limit; prints one JSON line per
instance (status, nodes, unit props) and a summary.  Sizes fixtures for
tests/golden/make_fullsolve.py (the oracle runs ~3 k nodes/s on 5-SAT n=200).

    python tools/fullsolve_probe.py <n> <m> <k> <seed> <count> [time_limit_s] [helpers_per_cu]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sat-mpi-stana-andrei_amd"))

import torch  # noqa: E402,F401

from satmi import _capi, cnf  # noqa: E402
from satmi.dpll import dpll_batch  # noqa: E402


def main():
    n, m, k, seed, count = (int(x) for x in sys.argv[1:6])
    tl = float(sys.argv[6]) if len(sys.argv) > 6 else 60.0
    helpers = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    _capi.set_split(_capi.SPLIT_ALWAYS, helpers)
    b = cnf.uniform_ksat(count, n, m, k, seed=seed)
    t0 = time.perf_counter()
    r = dpll_batch(b, mode="sound", max_solutions=1, time_limit=tl)
    dt = time.perf_counter() - t0
    rows = []
    for i in range(count):
        c = r.counter_dict(i)
        rows.append({"i": i, "status": int(r.status[i]), "sat": int(c["solutions"] > 0), "nodes": c["nodes"],
                     "unit_props": c["unit_props"]})
        print(json.dumps(rows[-1]), flush=True)
    done = [x for x in rows if x["status"] in (0, 1)]
    print(json.dumps({"n": n, "m": m, "k": k, "seed": seed, "count": count, "time_limit": tl, "wall_s": dt,
                      "decided": len(done), "sat": sum(x["sat"] for x in done),
                      "nodes_sorted": sorted(x["nodes"] for x in done)}), flush=True)


if __name__ == "__main__":
    main()
