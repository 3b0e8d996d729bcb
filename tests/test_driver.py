"""The comparison / report driver (satmi/driver.py) on CPU: the report format
against a block of the reference's own rezultat.txt (tests/golden/
rezultat_block.txt), result strings, the deadline mapping, and a scripted menu
session on stub solvers (the real solvers need the GPU: tests/test_driver_gpu.py)."""
import os

import pytest

from satmi import driver
from satmi.solvers import SolverTimeout


def _formula_50x10():
    # 50 clauses over 10 variables with 305 literals: the statistics of the fixture block
    return ([[(i + j) % 10 + 1 for j in range(6)] for i in range(45)] +
            [[(i + j) % 10 + 1 for j in range(7)] for i in range(5)])


def test_report_matches_reference_block(tmp_path, monkeypatch, golden_dir):
    with open(os.path.join(golden_dir, "rezultat_block.txt")) as fh:
        expected = fh.read()
    monkeypatch.setattr(driver.time, "strftime", lambda fmt: "2025-05-10 14:54:22")
    results = {
        "Resolution": {"time": 60, "memory": 722.88, "output": "Timeout after 60 seconds"},
        "Davis-Putnam": {"time": 0.109294, "memory": 31.44, "output": "Formula is satisfiable"},
        "DPLL": {"time": 60, "memory": 31.12, "output": "Timeout after 60 seconds"},
        "PySAT": {"time": 0.10798, "memory": 31.0,
                  "output": "Found 1 solution(s)\nFirst assignment sample: {1: False, 2: True, 3: False}..."},
        "Hybrid": {"time": 60, "memory": 31.02, "output": "Timeout after 60 seconds"},
    }
    out = tmp_path / "rezultat.txt"
    said = []
    driver.save_results_to_file(_formula_50x10(), results, str(out), print_fn=said.append)
    assert out.read_text() == expected
    assert said == [f"\nResults saved to {out} (without clause details)"]
    driver.save_results_to_file(_formula_50x10(), results, str(tmp_path), print_fn=said.append)
    assert said[-1].startswith("Error saving file:")


def test_describe_result():
    assert driver.describe_result("Resolution", False) == "Formula is unsatisfiable"
    assert driver.describe_result("Davis-Putnam", True) == "Formula is satisfiable"
    assert driver.describe_result("DPLL", []) == "No solutions found"
    assert driver.describe_result("DPLL", [{1: True, 2: False}, {1: False}]) == \
        "Found 2 solution(s)\nFirst assignment sample: {1: True, 2: False}..."
    assert driver.describe_result("CDCL", (True, {3: True})) == "Formula is satisfiable\nAssignment sample: {3: True}..."


def test_execute_with_timeout_maps_deadlines_and_errors():
    def late(f):
        raise SolverTimeout("deadline")

    def broken(f):
        raise ValueError("bad formula")

    assert driver.execute_with_timeout(lambda f: len(f), [[1]], 60) == (1, None)
    assert driver.execute_with_timeout(late, [[1]], 60) == (None, "Timeout after 60 seconds")
    assert driver.execute_with_timeout(broken, [[1]], 60) == (None, "bad formula")


def test_read_formula_from_input():
    feed = iter(["1 -2 0", "3", "x", "0 1 0", "2 0", "done"])
    printed = []
    f = driver.read_formula_from_input(lambda prompt: next(feed), printed.append)
    assert f == [[1, -2], [2]]
    assert "Error: Clause must end with 0" in printed and "Error: Please enter integers only" in printed
    assert "Error: 0 can only appear at end of clause" in printed


def test_scripted_menu_session(tmp_path):
    def failing(formula):
        raise RuntimeError("boom")

    table = {"1": ("Resolution", lambda f: False), "3": ("DPLL", lambda f: [{1: True}]),
             "4": ("CDCL", failing)}
    feed = iter(["1", "1 0", "-1 0", "done", "7", "y", "2", "3"])
    printed = []
    report = tmp_path / "rezultat.txt"
    driver.main_menu(lambda prompt: next(feed), printed.append, solver_table=table, report_file=str(report))
    text = report.read_text()
    assert "Resolution" in text and "Formula is unsatisfiable" in text
    assert "Found 1 solution(s)" in text
    assert "CDCL            Error        " in text   # a failing solver is reported as an error row
    assert printed[-1] == "Exiting program."


def _pipe_fixture(golden_dir):
    import json
    with open(os.path.join(golden_dir, "driver_pipe.json")) as fh:
        return json.load(fh)


def test_large_results_time_out_like_the_reference_queue(golden_dir):
    """REF.py:417-431 joins its solver child before draining the result queue,
    so a result whose pickle does not fit the pipe reads as a timeout there.
    Pinned by running the reference's own execute_with_timeout
    (tests/golden/make_golden_pipe.py): the exact byte boundary on stub
    results, and REF-mode DPLL results (here from the oracle, REF.py:133-214)
    either side of it -- same pickled size, same outcome."""
    import oracle
    fx = _pipe_fixture(golden_dir)
    assert driver.pipe_capacity() == fx["pipe_buffer_bytes"]
    assert any(c["outcome"] == "result" for c in fx["stub_cases"])
    assert any(c["outcome"] != "result" for c in fx["stub_cases"])
    for c in fx["stub_cases"]:
        got = driver.execute_with_timeout(lambda f, n=c["string_len"]: "x" * n, [[1]], 60)
        want = ("x" * c["string_len"], None) if c["outcome"] == "result" else (None, "Timeout after 60 seconds")
        assert got == want, c["payload_bytes"]
    outcomes = set()
    for c in fx["cases"]:
        sols = oracle.dpll(c["formula"], "ref")["solutions"]
        result = [{abs(l): l > 0 for l in s} for s in sols]
        assert len(result) == c["solutions"]
        got = driver.execute_with_timeout(lambda f: result, c["formula"], 60)
        if c["outcome"] == "result":
            assert got == (result, None)
        else:
            assert got == (None, c["outcome"].format(timeout=60))
        from multiprocessing.reduction import ForkingPickler
        assert len(ForkingPickler.dumps(("result", result))) == c["payload_bytes"]
        outcomes.add(c["outcome"])
    assert len(outcomes) == 2
    # the opt-out returns the result itself
    big = [{i: True} for i in range(1, 20001)]
    driver.REFERENCE_PIPE_LIMIT = False
    try:
        assert driver.execute_with_timeout(lambda f: big, [[1]], 60) == (big, None)
    finally:
        driver.REFERENCE_PIPE_LIMIT = True
    assert driver.execute_with_timeout(lambda f: big, [[1]], 60) == (None, "Timeout after 60 seconds")
