"""CPU baseline on all host cores: the oracle's SOUND-mode DPLL (oracle/sat_oracle.c,
a C restatement of REF.py:133-214) over a sample of the bench batch, one worker
process per core.

TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg runs this file as a CHILD
PROCESS (it never imports torch and never touches the GPU), so the worker pool
is forked from a process with no HIP state.

    python oracle/cpu_pool.py <batch_dir> <seconds> <node_limit> <workers>

<batch_dir> holds icb.npy / clb.npy / lits.npy (the CSR arrays of include/satmi.h),
memory-mapped by every worker.

Worker w solves instances w, w + workers, w + 2*workers, ... of the sample until
`seconds` pass; prints one JSON line: instances and unit-props per second over
the slowest worker's wall time.
"""
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle  # noqa: E402


def _instance(icb, clb, lits, b):
    c0, c1 = int(icb[b]), int(icb[b + 1])
    return [lits[clb[c]:clb[c + 1]].tolist() for c in range(c0, c1)]


def _worker(args):
    path, seconds, node_limit, w, workers = args
    icb, clb, lits = (np.load(os.path.join(path, f + ".npy"), mmap_mode="r") for f in ("icb", "clb", "lits"))
    B = icb.shape[0] - 1
    oracle.lib()
    t0 = time.perf_counter()
    done = props = 0
    for b in range(w, B, workers):
        r = oracle.dpll(_instance(icb, clb, lits, b), "sound", max_solutions=1, sol_cap=1, node_limit=node_limit)
        props += r["counters"]["unit_props"]
        done += 1
        if time.perf_counter() - t0 > seconds:
            break
    return done, props, time.perf_counter() - t0


def run(path, seconds, node_limit, workers):
    oracle.lib()   # build once before forking
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        res = pool.map(_worker, [(path, seconds, node_limit, w, workers) for w in range(workers)])
    done = sum(r[0] for r in res)
    props = sum(r[1] for r in res)
    wall = max(r[2] for r in res)
    return {"instances": done, "unit_props": props, "seconds": wall, "workers": workers,
            "instances_per_s": done / wall, "unit_props_per_s": props / wall}


if __name__ == "__main__":
    p, s, nl, wk = sys.argv[1], float(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    print(json.dumps(run(p, s, nl, wk)), flush=True)
