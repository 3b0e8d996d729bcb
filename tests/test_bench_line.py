"""bench.py's printed line stays parseable: main()'s JSON assembly
(compact_line) on stub legs is under LINE_BUDGET bytes and keeps every key of
the driver's contract, the headline's full roofline / issue roofline / CPU
baseline, and each leg's figures (CPU only, no GPU).

The stubs are the r05 final line (profiles/r05/final/bench.json: 25 KB
uncompacted, the line the driver could not parse) with every leg of
bench.LEGS filled from its largest leg."""
import copy
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _full_line():
    with open(os.path.join(ROOT, "profiles", "r05", "final", "bench.json")) as fh:
        full = json.load(fh)
    biggest = max(full["configs"].values(), key=lambda r: len(json.dumps(r)))
    for name, _, _ in bench.LEGS:   # every leg this bench runs, each as large as the largest r05 leg
        full["configs"].setdefault(name, copy.deepcopy(biggest))
    return full


def test_compact_line_fits_the_budget():
    full = _full_line()
    assert len(json.dumps(full)) > bench.LINE_BUDGET   # the stub is a real oversized line
    line = json.dumps(bench.compact_line(full))
    assert len(line.encode()) < bench.LINE_BUDGET, len(line)
    assert "\n" not in line


def test_compact_line_keeps_the_contract_and_the_headline_figures():
    full = _full_line()
    c = bench.compact_line(full)
    for k in CONTRACT:
        assert k in c, k
    for k in ("value", "ms_per_step", "steps", "warmup", "n_gpus"):
        assert c[k] == full[k], k   # the headline's own numbers unrounded
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in c["roofline"], k
    assert abs(c["roofline"]["frac"] / full["roofline"]["frac"] - 1) < 1e-3
    for k in ("bound", "frac", "fracs", "stale"):
        assert k in c["roofline_issue"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c["cpu_baseline"], k
    assert set(c["configs"]) == set(full["configs"])
    for name, leg in c["configs"].items():
        for k in ("value", "unit", "ms_per_step", "steps", "roofline", "cpu_baseline"):
            assert k in leg, (name, k)
        assert abs(leg["value"] / full["configs"][name]["value"] - 1) < 1e-3


def test_compact_line_without_legs_or_baseline():
    full = _full_line()
    for k in ("configs", "configs_note", "roofline_issue", "cpu_baseline", "branch_split"):
        full.pop(k, None)
    c = bench.compact_line(full)
    assert "configs" not in c and c.get("cpu_baseline") is None
    json.dumps(c)


def test_cpu_baseline_is_scaled_only_when_asked():
    """configs[2] / configs[1] time instances the oracle actually solves: the
    node-capped, scaled sample is the uf250-solved leg's alone (--cpu-scaled)."""
    assert not bench.parse([]).cpu_scaled
    assert not bench.parse(["--workload", "3sat-n50"]).cpu_scaled
    scaled = [name for name, _, extra in bench.LEGS if "--cpu-scaled" in extra]
    assert scaled and all("solved" in name for name in scaled)
