"""Golden vectors at the configs[3] BENCH sizes, from the REFERENCE's own solvers.

Run here (the container that holds /root/reference):
    python tests/golden/make_golden_bench.py            # both fixtures
    python tests/golden/make_golden_bench.py res|dp     # one of them

* `resolution_php43.json` -- REF.py:63-95 `resolution_solver` on PHP(4,3)
  (the `php-res` bench workload), observed until its 4th saturation pass: the
  new-clause SET of every pass (REF.py:94's `seen.update(new_clauses)`).  The
  run is stopped right after the 4th pass by raising a sentinel from the
  observer (the 5th pass is 1.6e10 pairs).  Passes 1-3 are stored in full;
  pass 4 (163,954 clauses) as its size plus the sha256 of its canonical form
  (every clause sorted, the clauses sorted, compact JSON) -- exact, and 60x
  smaller than the clause list.
* `dp_php65.json` -- REF.py:98-130 `davis_putnam_solver` on PHP(6,5) (the
  `php-dp` bench workload) to the end: per elimination step the variable
  popped (REF.py:103) and the clause list after it (REF.py:127) with each
  clause set in CPython's iteration order -- stored as its length, its
  literal count and the sha256 of its compact JSON form (the full lists of
  the first steps too), plus the verdict.

The reference functions are loaded exactly as make_golden.py does (ast-extracted,
executed unmodified, PySAT import skipped -- no stand-in); the observers are
read-only: `sys.setprofile` for resolution (only C-function calls fire, so the
27.8 M pair iterations of pass 4 run untraced), a line tracer restricted to the
Davis-Putnam frame for DP.  Plain-data JSON only; no reference source text.
"""
import hashlib
import json
import os
import sys
import time

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import make_golden as mg  # noqa: E402  (loads the reference functions)

OUT_DIR = os.path.dirname(os.path.abspath(__file__))


def canon_sha(clauses):
    """sha256 of a clause SET: each clause sorted, then the clauses sorted."""
    s = json.dumps(sorted(sorted(c) for c in clauses), separators=(",", ":"))
    return hashlib.sha256(s.encode()).hexdigest()


def list_sha(clauses):
    """sha256 of an ORDERED clause list (clause order and literal order kept)."""
    s = json.dumps([list(c) for c in clauses], separators=(",", ":"))
    return hashlib.sha256(s.encode()).hexdigest()


class _Stop(Exception):
    pass


def resolution_php43(passes=4, full_passes=3):
    fn = mg.NS["resolution_solver"]
    code_res = fn.__code__
    got = []

    def prof(frame, event, arg):
        # REF.py:94 `seen.update(new_clauses)` is the only `update` call the
        # resolution frame makes; its operand is the pass's new-clause set.
        if event == "c_call" and frame.f_code is code_res and getattr(arg, "__name__", "") == "update":
            got.append([sorted(c) for c in frame.f_locals["new_clauses"]])
            if len(got) == passes:
                raise _Stop()

    f = mg.pigeonhole(3)
    t = time.time()
    sys.setprofile(prof)
    try:
        res = fn([list(c) for c in f])
    except _Stop:
        res = None
    finally:
        sys.setprofile(None)
    dt = time.time() - t
    assert res is None and len(got) == passes, (res, len(got))
    out = []
    for k, p in enumerate(got):
        e = {"pass": k + 1, "count": len(p), "sha256": canon_sha(p)}
        if k < full_passes:
            e["clauses"] = sorted(sorted(c) for c in p)
        out.append(e)
    return {"formula": f, "holes": 3, "passes_observed": passes, "stopped_after_pass": passes,
            "result": None, "passes": out, "reference_seconds": round(dt, 1)}


def dp_php65(full_steps=4):
    fn = mg.NS["davis_putnam_solver"]
    code_dp = fn.__code__
    steps = []

    def local(frame, event, arg):
        if event == "line":
            ln = frame.f_lineno
            if ln == mg.L_DP_POS:
                steps.append({"var": frame.f_locals["var"]})
            elif ln == mg.L_DP_VARS and steps and "n" not in steps[-1]:
                cl = frame.f_locals["clauses"]
                lst = [list(c) for c in cl]
                s = steps[-1]
                s["n"] = len(lst)
                s["lits"] = sum(len(c) for c in lst)
                s["sha256"] = list_sha(lst)
                if len(steps) <= full_steps:
                    s["clauses"] = lst
        return local

    def glob(frame, event, arg):
        if event == "call" and frame.f_code is code_dp:
            return local
        return None

    f = mg.pigeonhole(5)
    t = time.time()
    sys.settrace(glob)
    try:
        res = fn([list(c) for c in f])
    finally:
        sys.settrace(None)
    dt = time.time() - t
    return {"formula": f, "holes": 5, "result": bool(res), "steps": steps, "reference_seconds": round(dt, 1)}


def main():
    which = sys.argv[1:] or ["res", "dp"]
    meta = {"generator": "tests/golden/make_golden_bench.py", "python": sys.version.split()[0],
            "reference": os.path.basename(mg.REF_FILE)}
    if "res" in which:
        c = resolution_php43()
        with open(os.path.join(OUT_DIR, "resolution_php43.json"), "w") as fh:
            json.dump({"meta": meta, "cases": [c]}, fh, separators=(",", ":"))
        print("resolution_php43", [p["count"] for p in c["passes"]], c["reference_seconds"], "s")
    if "dp" in which:
        c = dp_php65()
        with open(os.path.join(OUT_DIR, "dp_php65.json"), "w") as fh:
            json.dump({"meta": meta, "cases": [c]}, fh, separators=(",", ":"))
        print("dp_php65", c["result"], len(c["steps"]), "steps", c["reference_seconds"], "s")


if __name__ == "__main__":
    main()
