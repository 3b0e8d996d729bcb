"""The comparison driver end to end on the GPU solvers: a scripted menu session
(REF.py:491-632) whose saved report carries the verdicts the reference's own
solvers give for the same formula (the oracle restates them)."""
import pytest

import oracle
from satmi import driver

pytestmark = pytest.mark.gpu


def test_menu_session_on_gpu_solvers(tmp_path):
    formula_lines = ["1 2 0", "-1 2 0", "1 -2 0", "-1 -2 0", "3 -4 0"]
    feed = iter(["1"] + formula_lines + ["done", "1,2,3,6", "y", "2", "3"])
    printed = []
    report = tmp_path / "rezultat.txt"
    driver.main_menu(lambda prompt: next(feed), printed.append, report_file=str(report))
    text = report.read_text()
    f = [[int(x) for x in line.split()[:-1]] for line in formula_lines]
    res = oracle.resolution(f)["result"]
    dp = oracle.dp(f)["result"]
    want_res = "Formula is " + ("satisfiable" if res == 1 else "unsatisfiable")
    want_dp = "Formula is " + ("satisfiable" if dp == 1 else "unsatisfiable")
    rows = {line[:15].strip(): line for line in text.splitlines() if line[:15].strip() in
            ("Resolution", "Davis-Putnam", "DPLL", "Hybrid")}
    assert want_res in rows["Resolution"] and want_dp in rows["Davis-Putnam"]
    nsol = len(oracle.dpll(f, "ref")["solutions"])
    want = f"Found {nsol} solution(s)" if nsol else "No solutions found"
    assert want in rows["DPLL"] and want in rows["Hybrid"]
    assert "- Clauses: 5" in text and "- Variables: 4" in text


def test_menu_large_formula_times_out_like_reference():
    """rezultat.txt:248-262: on the 1000-clause menu formula (avg length ~50,
    100 variables) the reference's DPLL and Hybrid rows read "Timeout after 60
    seconds".  The GPU drop-in runs the same enumeration (wide kernel: the
    image exceeds one wave's LDS) and reports the same timeout row, here with a
    2-second deadline."""
    import random

    from satmi.solvers import dpll_optimized, generate_large_formula, hybrid_solver
    random.seed(1100)
    f = generate_large_formula(1000, 100, 100)
    results = driver.run_solvers(f, [("DPLL", dpll_optimized), ("Hybrid", hybrid_solver)], timeout=2,
                                 print_fn=lambda *a: None)
    for name in ("DPLL", "Hybrid"):
        assert results[name]["output"] == "Timeout after 2 seconds", results[name]
        assert results[name]["time"] == 2


def test_large_results_time_out_like_the_reference_queue_on_gpu(golden_dir):
    """The GPU dpll_optimized through the driver: results the reference's
    result pipe cannot carry read as its timeout, the others come back whole
    (tests/golden/driver_pipe.json, from REF.py's own execute_with_timeout)."""
    import json
    import os
    from satmi.solvers import dpll_optimized
    with open(os.path.join(golden_dir, "driver_pipe.json")) as fh:
        fx = json.load(fh)
    for c in fx["cases"]:
        result, error = driver.execute_with_timeout(dpll_optimized, c["formula"], 60)
        if c["outcome"] == "result":
            assert error is None and len(result) == c["solutions"], c["shape"]
            sols = oracle.dpll(c["formula"], "ref")["solutions"]
            assert result == [{abs(l): l > 0 for l in s} for s in sols]
        else:
            assert (result, error) == (None, c["outcome"].format(timeout=60)), c["shape"]
