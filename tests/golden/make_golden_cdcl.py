"""Golden vectors for CDCL by running the REFERENCE's own CDCLSolver class.

Run here (the container that holds /root/reference):
    python tests/golden/make_golden_cdcl.py

* Parses the reference script with `ast` and executes only its own definitions
  of generate_large_formula and the CDCLSolver class (REF.py:21-29, :217-379),
  unmodified (the PySAT import, REF.py:6-7, is not executed; CDCL does not use it).
* The reference's solve loop (REF.py:247-267) has no bound of its own -- its
  caller kills it after 60 s (REF.py:417-437) -- so a read-only `sys.settrace`
  observer counts the loop's propagate() calls and stops the run by raising
  at the call that would start iteration `max_iter + 1`.  It also counts
  analyze_conflict calls (conflicts), select_variable calls that returned a
  variable (decisions) and learn_clause calls with a non-empty clause.
* Records per formula: the verdict (1 True, 0 False, -1 stopped at max_iter,
  -2 the reference raised), the assignment dict in its insertion order (the
  returned model, or the live dict where the run was stopped), the decision
  level, var_inc, the formula's final length and the watch-list key count.
  Plain-data JSON only; no reference source text is stored.
"""
import ast
import json
import os
import random
import sys

sys.dont_write_bytecode = True

REF_FILE = "/root/reference/comparatie intre algoritmii de rezolvare a seturilor de clauze.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cdcl_ref.json")


def load_reference():
    tree = ast.parse(open(REF_FILE, encoding="utf-8").read())
    body = []
    for node in tree.body:
        if isinstance(node, ast.Import):
            body.append(node)
        elif isinstance(node, ast.ImportFrom) and not node.module.startswith("pysat"):
            body.append(node)
        elif isinstance(node, ast.Assign):
            body.append(node)
        elif isinstance(node, ast.FunctionDef) and node.name == "generate_large_formula":
            body.append(node)
        elif isinstance(node, ast.ClassDef) and node.name == "CDCLSolver":
            body.append(node)
    ns = {"__name__": "reference_cdcl"}
    exec(compile(ast.Module(body=body, type_ignores=[]), REF_FILE, "exec"), ns)
    return ns


NS = load_reference()


class Stop(Exception):
    pass


def run_cdcl(formula, max_iter):
    solver_cls = NS["CDCLSolver"]
    codes = {name: getattr(solver_cls, name).__code__
             for name in ("propagate", "analyze_conflict", "select_variable", "learn_clause")}
    obs = {"iterations": 0, "conflicts": 0, "decisions": 0, "learned": 0}

    def tracer(frame, event, arg):
        co = frame.f_code
        if event == "call":
            if co is codes["propagate"]:
                if obs["iterations"] >= max_iter:
                    raise Stop()
                obs["iterations"] += 1
            elif co is codes["analyze_conflict"]:
                obs["conflicts"] += 1
            elif co is codes["learn_clause"] and frame.f_locals["clause"]:
                obs["learned"] += 1
            return tracer if co is codes["select_variable"] else None
        if event == "return" and co is codes["select_variable"] and arg is not None:
            obs["decisions"] += 1
        return None

    f_copy = [list(c) for c in formula]
    solver = None
    sys.settrace(tracer)
    try:
        solver = solver_cls(f_copy)   # cdcl_solve (REF.py:382-384)
        sat, model = solver.solve()
        result = 1 if sat else 0
    except Stop:
        result, model = -1, None
    except Exception as e:  # noqa: BLE001 - the reference's own error (e.g. KeyError)
        result, model = -2, None
        obs["error"] = type(e).__name__
    finally:
        sys.settrace(None)
    live = model if model is not None else (solver.assignment if solver is not None else {})
    return {
        "formula": formula, "max_iter": max_iter, "result": result,
        "assignment": [v if b else -v for v, b in live.items()],
        "level": solver.level if solver is not None else 0,
        "var_inc": solver.var_inc if solver is not None else 1.0,
        "clauses": len(f_copy), "watch_keys": len(solver.watch_list) if solver is not None else 0,
        "stats": obs,
    }


def uniform_ksat(rng, n, m, k):
    return [[v if rng.random() < 0.5 else -v for v in rng.sample(range(1, n + 1), k)] for _ in range(m)]


def pigeonhole(holes):
    f = []
    for p in range(holes + 1):
        f.append([p * holes + h + 1 for h in range(holes)])
    for h in range(holes):
        for p in range(holes + 1):
            for q in range(p + 1, holes + 1):
                f.append([-(p * holes + h + 1), -(q * holes + h + 1)])
    return f


def main():
    cases = []
    edge = [[], [[]], [[1]], [[1], [-1]], [[1, -1]], [[1, 1]], [[-1, -2]], [[1, 2], [-1, 2], [1, -2], [-1, -2]],
            [[1], [2, 3]], [[2], [-2, 1], [-1]], [[1, 2, 3], [], [-3]], [[3, -3, 2], [-2]]]
    for f in edge:
        cases.append(dict(run_cdcl(f, 400), tag="edge"))
    # the reference's own menu generator, rezultat.txt-sized runs (5..80 clauses)
    for seed, (nc, ml, nv) in enumerate([(5, 3, 3), (8, 5, 5), (9, 6, 6), (10, 5, 7), (12, 4, 6), (20, 5, 8),
                                         (30, 6, 10), (80, 12, 15), (40, 3, 12), (60, 4, 14)] * 3):
        random.seed(1000 + seed)
        f = NS["generate_large_formula"](nc, ml, nv)
        cases.append(dict(run_cdcl(f, 600), tag="menu"))
    rng = random.Random(7)
    for i in range(120):
        n = rng.randint(3, 14)
        m = rng.randint(1, 5 * n)
        k = rng.randint(1, min(4, n))
        cases.append(dict(run_cdcl(uniform_ksat(rng, n, m, k), 300), tag="random"))
    for holes in (1, 2, 3):
        cases.append(dict(run_cdcl(pigeonhole(holes), 500), tag="php"))
    with open(OUT, "w") as fh:
        json.dump({"source": "REF.py CDCLSolver (REF.py:217-379), run by tests/golden/make_golden_cdcl.py",
                   "cases": cases}, fh, separators=(",", ":"))
    by = {}
    for c in cases:
        by[c["result"]] = by.get(c["result"], 0) + 1
    print(f"{len(cases)} cases -> {OUT}; results {by}")


if __name__ == "__main__":
    main()
