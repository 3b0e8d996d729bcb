"""CPU baselines on all host cores: the oracle (oracle/*.c, C restatements of
REF.py's solvers) over a sample of a bench workload, one worker process per core.

TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline legs run this file as a CHILD
PROCESS (it never imports torch and never touches the GPU), so the worker pool
is forked from a process with no HIP state.

    python oracle/cpu_pool.py <kind> <batch_dir> <seconds> <param> <workers>

<batch_dir> holds icb.npy / clb.npy / lits.npy (the CSR arrays of include/satmi.h),
memory-mapped by every worker.  Kinds:
    dpll  SOUND-mode DPLL (REF.py:133-214), <param> = node limit (0: none);
          worker w solves instances w, w + workers, ... of the sample
    cdcl  cdcl_solve (REF.py:217-384), <param> = max_iter; instances as dpll
    dp    Davis-Putnam (REF.py:98-130) of instance 0, repeated (replicas)
    res   resolution (REF.py:63-95) of instance 0, <param> = passes, repeated;
          the unit is derived clauses
    resset / dpset  resolution / Davis-Putnam of every instance to the end,
          worker w solving instances w, w + workers, ... and cycling over the
          set until the time is up; the unit is formulas
until `seconds` pass (every worker finishes at least one unit).  Prints one
JSON line: units and unit-props (dpll) per second over the slowest worker's
wall time.
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


def _solve(kind, f, param):
    """(units, unit-props) of one oracle call."""
    if kind == "dpll":
        r = oracle.dpll(f, "sound", max_solutions=1, sol_cap=1, node_limit=param)
        return 1, r["counters"]["unit_props"]
    if kind == "cdcl":
        oracle.cdcl(f, max_iter=param)
        return 1, 0
    if kind == "dp":
        oracle.dp(f)
        return 1, 0
    if kind == "res":
        return sum(oracle.resolution(f, max_passes=param)["pass_new"]), 0
    if kind == "resset":
        oracle.resolution(f)
        return 1, 0
    if kind == "dpset":
        oracle.dp(f)
        return 1, 0
    raise ValueError(kind)


def _worker(args):
    kind, path, seconds, param, w, workers = args
    icb, clb, lits = (np.load(os.path.join(path, f + ".npy"), mmap_mode="r") for f in ("icb", "clb", "lits"))
    B = icb.shape[0] - 1
    oracle.lib()
    t0 = time.perf_counter()
    done = props = 0
    if B <= 0:
        return done, props, time.perf_counter() - t0
    replicas = kind in ("dp", "res")
    cycle = kind in ("resset", "dpset")
    f0 = _instance(icb, clb, lits, 0) if replicas else None
    # the sample's instances are solved once each, except by the cycling kinds:
    # a worker past the sample's end has nothing to do (it must not solve and
    # count an instance another worker already counted)
    b = w % B if cycle else w
    while replicas or cycle or b < B:
        u, p = _solve(kind, f0 if replicas else _instance(icb, clb, lits, b), param)
        done += u
        props += p
        b += workers
        if cycle:
            b %= B
        if time.perf_counter() - t0 > seconds:
            break
    return done, props, time.perf_counter() - t0


def run(kind, path, seconds, param, workers):
    oracle.lib()   # build once before forking
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        res = pool.map(_worker, [(kind, path, seconds, param, w, workers) for w in range(workers)])
    done = sum(r[0] for r in res)
    props = sum(r[1] for r in res)
    wall = max(r[2] for r in res)
    return {"kind": kind, "units": done, "instances": done, "unit_props": props, "seconds": wall,
            "workers": workers, "units_per_s": done / wall, "instances_per_s": done / wall,
            "unit_props_per_s": props / wall}


if __name__ == "__main__":
    k, p, s, prm, wk = sys.argv[1], sys.argv[2], float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    print(json.dumps(run(k, p, s, prm, wk)), flush=True)
