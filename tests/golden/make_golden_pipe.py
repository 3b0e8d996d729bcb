"""Pin the reference driver's large-result behaviour (REF.py:408-437).

Run here (the container that holds /root/reference):
    python tests/golden/make_golden_pipe.py

REF.py's execute_with_timeout starts the solver in a child process, JOINS the
child (REF.py:423) and only then drains the result queue (REF.py:430-431).  The
child's queue feeder writes the pickled ('result', value) into a pipe; when it
does not fit the pipe's buffer the write blocks until someone reads, so the
child never exits, the join times out and the reference reports "Timeout after
N seconds" for a solver that had finished.  satmi/driver.py reproduces that
outcome (without the wait).  This script runs the reference's OWN
run_solver_with_timeout / execute_with_timeout / dpll_optimized /
generate_large_formula (executed from REF.py's source via `ast`, PySAT import
skipped, nothing else defined) on menu-shaped formulas whose REF-mode DPLL
results straddle the pipe size, and records per formula: the formula, the
number of solutions, the pickled size of ('result', solutions) and what the
reference's execute_with_timeout returned (result or timeout message).

Fixture: tests/golden/driver_pipe.json (data only).
"""
import ast
import fcntl
import json
import os
import random
import sys
import time
from multiprocessing.reduction import ForkingPickler

sys.dont_write_bytecode = True

REF_FILE = "/root/reference/comparatie intre algoritmii de rezolvare a seturilor de clauze.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "driver_pipe.json")
WANTED = ("generate_large_formula", "dpll_optimized", "run_solver_with_timeout", "execute_with_timeout")
TIMEOUT = 4   # seconds the reference waits (its menu uses 60; the outcome does not depend on it)


def load_reference():
    tree = ast.parse(open(REF_FILE, encoding="utf-8").read())
    body = [n for n in tree.body
            if isinstance(n, ast.Import) or (isinstance(n, ast.ImportFrom) and not n.module.startswith("pysat"))
            or isinstance(n, ast.Assign) or (isinstance(n, ast.FunctionDef) and n.name in WANTED)]
    ns = {"__name__": "reference_functions"}
    exec(compile(ast.Module(body=body, type_ignores=[]), REF_FILE, "exec"), ns)
    return ns


def pipe_size():
    r, w = os.pipe()
    try:
        return fcntl.fcntl(w, 1032)   # F_GETPIPE_SZ
    finally:
        os.close(r)
        os.close(w)


def main():
    ns = load_reference()
    cases = []
    # (clauses, max literals, variables, seed): rezultat.txt-style menu shapes
    # whose REF-mode result sizes fall on both sides of the pipe buffer
    # (found by scanning seeds: REF-mode results come in powers of two)
    shapes = [(50, 7, 10, 0), (50, 7, 10, 3), (30, 10, 12, 6), (30, 10, 12, 3), (30, 10, 12, 2),
              (25, 10, 15, 56), (25, 10, 15, 42), (30, 10, 12, 24), (12, 6, 13, 1), (25, 10, 15, 29),
              (30, 10, 12, 7)]
    for ncl, maxlit, nv, seed in shapes:
        random.seed(seed)
        formula = ns["generate_large_formula"](ncl, maxlit, nv)
        t = time.time()
        direct = ns["dpll_optimized"]([list(c) for c in formula])
        dt = time.time() - t
        if dt > 2.0:
            continue
        payload = len(ForkingPickler.dumps(("result", direct)))
        result, error = ns["execute_with_timeout"](ns["dpll_optimized"], [list(c) for c in formula], TIMEOUT)
        cases.append({"shape": [ncl, maxlit, nv, seed], "formula": formula, "solutions": len(direct),
                      "payload_bytes": payload,
                      "outcome": "result" if error is None else error.replace(str(TIMEOUT), "{timeout}"),
                      "result_matches_direct": (result == direct) if error is None else None})
        print(ncl, maxlit, nv, seed, len(direct), payload, cases[-1]["outcome"], flush=True)
    # the boundary itself: a stub solver returning a string whose pickled
    # ('result', value) is a few bytes either side of the pipe buffer
    stubs = []
    cap = pipe_size()
    for want in range(cap - 8, cap + 1):
        n = want
        while len(ForkingPickler.dumps(("result", "x" * n))) > want:
            n -= 1
        if len(ForkingPickler.dumps(("result", "x" * n))) != want:
            continue
        result, error = ns["execute_with_timeout"](lambda f, n=n: "x" * n, [[1]], TIMEOUT)
        stubs.append({"string_len": n, "payload_bytes": want,
                      "outcome": "result" if error is None else error.replace(str(TIMEOUT), "{timeout}")})
        print("stub", n, want, stubs[-1]["outcome"], flush=True)
    json.dump({"source": "REF.py execute_with_timeout(dpll_optimized, formula, %d) run here" % TIMEOUT,
               "python": sys.version.split()[0], "pipe_buffer_bytes": pipe_size(),
               "pickle": "multiprocessing.reduction.ForkingPickler.dumps(('result', value)), default protocol",
               "cases": cases, "stub_cases": stubs}, open(OUT, "w"), indent=0)


if __name__ == "__main__":
    main()
