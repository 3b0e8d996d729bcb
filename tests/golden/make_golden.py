"""Generate golden vectors by running the REFERENCE's own solver functions.

Run here (the container that holds /root/reference):
    python tests/golden/make_golden.py

What it does
------------
* Parses the reference script with `ast` and executes *only* the reference's
  own definitions of generate_large_formula / resolution_solver /
  davis_putnam_solver / dpll_optimized (REF.py:21-214), unmodified.  The
  module-level `from pysat...` import (REF.py:6-7) is not executed: PySAT is a
  third-party dependency that is absent from this image and none of these four
  functions uses it.  No stand-in for it is written.
* Observes the reference while it runs with `sys.settrace` (read-only): per
  dpll_optimized call tree it counts calls (nodes), unit assignments
  (REF.py:154), pure-literal assignments (REF.py:189), branch assignments
  (REF.py:212) and conflicts (REF.py:169); for Davis-Putnam it records the
  eliminated variable and the clause list (with each clause set's CPython
  iteration order) after every elimination step; for resolution it records the
  new-clause set of every saturation pass.
* Writes plain-data JSON fixtures (inputs + observed outputs) next to this file.
  No reference source text is stored.

Bytecode caching is disabled so nothing is written under /root/reference.
"""
import ast
import json
import os
import random
import signal
import sys

sys.dont_write_bytecode = True

REF_FILE = "/root/reference/comparatie intre algoritmii de rezolvare a seturilor de clauze.py"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))
WANTED = ("generate_large_formula", "resolution_solver", "davis_putnam_solver", "dpll_optimized")


def load_reference():
    src = open(REF_FILE, encoding="utf-8").read()
    tree = ast.parse(src)
    body = []
    for node in tree.body:
        if isinstance(node, ast.Import):
            body.append(node)
        elif isinstance(node, ast.ImportFrom) and not node.module.startswith("pysat"):
            body.append(node)
        elif isinstance(node, ast.Assign):
            body.append(node)
        elif isinstance(node, ast.FunctionDef) and node.name in WANTED:
            body.append(node)
    ns = {"__name__": "reference_functions"}
    exec(compile(ast.Module(body=body, type_ignores=[]), REF_FILE, "exec"), ns)

    # locate the statements we observe, by their source text (no hard-coded numbers)
    lines = {}
    for fn in ast.walk(tree):
        if isinstance(fn, ast.FunctionDef) and fn.name in WANTED:
            for st in ast.walk(fn):
                if isinstance(st, (ast.Assign, ast.Return, ast.Expr)):
                    txt = ast.unparse(st)
                    lines.setdefault((fn.name, txt), []).append(st.lineno)
    return ns, lines


NS, LINES = load_reference()


def _line(fn, txt):
    ls = LINES[(fn, txt)]
    assert len(ls) == 1, (fn, txt, ls)
    return ls[0]


L_UNIT = _line("dpll_optimized", "a[var] = val")
L_PURE = _line("dpll_optimized", "new_assignment[abs(lit)] = lit > 0")
L_DEC = _line("dpll_optimized", "new_assignment[var] = val")
L_CONF = _line("dpll_optimized", "(formula, assignment) = unit_propagate(formula, assignment)") + 2  # 'return []'
L_DP_POS = _line("davis_putnam_solver", "pos_clauses = [c for c in clauses if var in c]")
# the statement appears twice (REF.py:100 and :128); the in-loop one is the later
L_DP_VARS = max(LINES[("davis_putnam_solver", "variables = {abs(lit) for clause in clauses for lit in clause}")])
L_RES_UPD = _line("resolution_solver", "seen.update(new_clauses)")


class Timeout(Exception):
    pass


def _alarm(signum, frame):
    raise Timeout()


def run_traced(fn_name, formula, seconds, *args):
    """Run a reference function on a deep copy of `formula` with a tracer."""
    fn = NS[fn_name]
    obs = {"nodes": 0, "unit_props": 0, "pure_assigns": 0, "decisions": 0, "conflicts": 0,
           "dp_steps": [], "res_passes": []}
    code_dpll = NS["dpll_optimized"].__code__
    code_dp = NS["davis_putnam_solver"].__code__
    code_res = NS["resolution_solver"].__code__
    # line numbers inside the source file; 'return []' after the unit_propagate call
    src_lines = open(REF_FILE, encoding="utf-8").read().splitlines()
    conf_line = None
    for ln in range(L_CONF - 2, L_CONF + 3):
        if src_lines[ln - 1].strip() == "return []":
            conf_line = ln
            break
    assert conf_line is not None

    def local_tracer(frame, event, arg):
        if event != "line":
            return local_tracer
        co = frame.f_code
        ln = frame.f_lineno
        if co is code_dp:
            if ln == L_DP_POS:
                obs["dp_steps"].append({"var": frame.f_locals["var"]})
            elif ln == L_DP_VARS and obs["dp_steps"] and "clauses" not in obs["dp_steps"][-1]:
                obs["dp_steps"][-1]["clauses"] = [list(c) for c in frame.f_locals["clauses"]]
        elif co is code_res:
            if ln == L_RES_UPD:
                nc = frame.f_locals["new_clauses"]
                obs["res_passes"].append(sorted(sorted(c) for c in nc))
        else:
            if ln == L_UNIT:
                obs["unit_props"] += 1
            elif ln == L_PURE:
                obs["pure_assigns"] += 1
            elif ln == L_DEC:
                obs["decisions"] += 1
            elif ln == conf_line and co is code_dpll:
                obs["conflicts"] += 1
        return local_tracer

    def global_tracer(frame, event, arg):
        if event == "call":
            co = frame.f_code
            if co is code_dpll:
                obs["nodes"] += 1
            if co.co_filename == REF_FILE:
                return local_tracer
        return None

    f_copy = [list(c) for c in formula]
    signal.signal(signal.SIGALRM, _alarm)
    signal.setitimer(signal.ITIMER_REAL, seconds)
    sys.settrace(global_tracer)
    try:
        result = fn(f_copy, *args)
    except Timeout:
        result = Timeout
    finally:
        sys.settrace(None)
        signal.setitimer(signal.ITIMER_REAL, 0)
    return result, obs


def dpll_case(formula, init=None, seconds=20.0):
    init_list = [] if init is None else [v if b else -v for v, b in init.items()]
    init_dict = None if init is None else dict(init)
    args = () if init_dict is None else (init_dict,)
    res, obs = run_traced("dpll_optimized", formula, seconds, *args)
    if res is Timeout:
        return None
    case = {
        "formula": formula,
        "init": init_list,
        "solutions": [[v if b else -v for v, b in sol.items()] for sol in res],
        "counters": {k: obs[k] for k in ("nodes", "unit_props", "pure_assigns", "decisions", "conflicts")},
    }
    if init_dict is not None:  # the caller's dict is mutated by the root unit_propagate (REF.py:167)
        case["init_after"] = [v if b else -v for v, b in init_dict.items()]
    return case


def dp_case(formula, seconds=20.0):
    res, obs = run_traced("davis_putnam_solver", formula, seconds)
    if res is Timeout:
        return None
    return {"formula": formula, "result": bool(res), "steps": obs["dp_steps"]}


def res_case(formula, seconds=20.0):
    res, obs = run_traced("resolution_solver", formula, seconds)
    if res is Timeout:
        return None
    return {"formula": formula, "result": bool(res), "passes": obs["res_passes"]}


def uniform_ksat(rng, n, m, k):
    out = []
    for _ in range(m):
        vs = rng.sample(range(1, n + 1), k)
        out.append([v if rng.random() < 0.5 else -v for v in vs])
    return out


def pigeonhole(holes):
    """PHP(holes+1, holes): var p*holes + h + 1 = pigeon p sits in hole h."""
    pig = holes + 1
    x = lambda p, h: p * holes + h + 1
    cls = [[x(p, h) for h in range(holes)] for p in range(pig)]
    for h in range(holes):
        for p in range(pig):
            for q in range(p + 1, pig):
                cls.append([-x(p, h), -x(q, h)])
    return cls


EDGE_FORMULAS = [
    [], [[]], [[1]], [[-1]], [[1], [-1]], [[1, -1]], [[1, 1]], [[1, 1], [-1]],
    [[1, 2], [-1, 2], [1, -2], [-1, -2]],
    [[1], [-1, 2], [-2, 3, 4]],
    [[1], [1], [-1, 2]],
    [[2], [1, -2], [-1, 3], [-3, -2]],
    [[1, 2, 3]], [[-1, -2], [-2, -3], [-1, -3]],
    [[1, 2], [], [3]],
    [[1, 2], [-2, 3], [-3, 1], [4, -4]],
    [[5, -3], [3, 1], [-1, -5, 2], [2, 4], [-4, -2, 3], [1]],
]


def main():
    rng = random.Random(20250614)
    dpll_cases, dp_cases, res_cases = [], [], []

    for f in EDGE_FORMULAS:
        for mk, lst in ((dpll_case, dpll_cases), (dp_case, dp_cases), (res_case, res_cases)):
            c = mk(f)
            if c is not None:
                lst.append(c)
    # caller-supplied initial assignments (REF.py:133-136)
    for f, init in (([[1, 2], [-1]], {2: False}), ([[1, 2], [-2, 3]], {3: False, 1: False}),
                    ([[1], [2, 3]], {1: True}), ([[-1, 2], [1, 3], [-3]], {4: True})):
        c = dpll_case(f, init)
        if c is not None:
            dpll_cases.append(c)

    # the reference's own generator (REF.py:21-29), driven by `random` as the script does
    for seed in range(60):
        random.seed(1000 + seed)
        nclauses = random.randint(3, 30)
        maxlit = random.randint(1, 5)
        nvars = random.randint(max(maxlit, 2), 9)
        f = NS["generate_large_formula"](nclauses, maxlit, nvars)
        c = dpll_case(f)
        if c is not None and len(c["solutions"]) <= 3000:
            dpll_cases.append(c)
        c = dp_case(f)
        if c is not None:
            dp_cases.append(c)
        if nclauses <= 14:
            c = res_case(f, seconds=5.0)
            if c is not None:
                res_cases.append(c)

    # uniform random 3-SAT near the threshold, small n (REF-mode enumeration stays small)
    for i in range(24):
        n = rng.randint(5, 10)
        m = int(round(4.26 * n))
        f = uniform_ksat(rng, n, m, 3)
        c = dpll_case(f)
        if c is not None:
            dpll_cases.append(c)
        c = dp_case(f)
        if c is not None:
            dp_cases.append(c)
    # larger DP cases: uniform 3-SAT n = 12..20 (verdicts pin the sound DPLL mode too)
    for i in range(40):
        n = rng.randint(12, 20)
        m = int(round(4.26 * n))
        f = uniform_ksat(rng, n, m, 3)
        c = dp_case(f, seconds=30.0)
        if c is not None:
            dp_cases.append(c)
    for holes in (1, 2, 3):
        c = dp_case(pigeonhole(holes))
        if c is not None:
            dp_cases.append(c)
    for holes in (1, 2):
        c = res_case(pigeonhole(holes), seconds=30.0)
        if c is not None:
            res_cases.append(c)
    # small random UNSAT-ish sets for resolution
    for i in range(20):
        n = rng.randint(3, 5)
        m = rng.randint(4, 9)
        f = uniform_ksat(rng, n, m, 2 if i % 2 else 3)
        c = res_case(f, seconds=5.0)
        if c is not None:
            res_cases.append(c)

    meta = {"generator": "tests/golden/make_golden.py", "python": sys.version.split()[0],
            "reference": os.path.basename(REF_FILE)}
    for name, cases in (("dpll_ref.json", dpll_cases), ("dp_ref.json", dp_cases), ("resolution_ref.json", res_cases)):
        with open(os.path.join(OUT_DIR, name), "w") as fh:
            json.dump({"meta": meta, "cases": cases}, fh, separators=(",", ":"))
        print(name, len(cases))


if __name__ == "__main__":
    main()
