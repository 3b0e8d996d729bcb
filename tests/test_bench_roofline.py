"""bench.py's roofline bookkeeping for the configs[3] legs (CPU only).

* php-res: the fused pass kernel (csrc/resolution.hip res_pass_packed_kernel)
  is charged against the issue pipe its SQ passes found binding
  (profiles/sq_issue.json "php-res_B1", per step) over the run's live kernel
  time, with the step's HBM bytes beside it;
* php-dp: a solve is a chain of dependent launches, priced against the
  launch rate of an empty chain of the same length measured on the GPU
  (satmi_launch_chain_floor; a fixed floor here)."""
import bench


def _res_stats(pair_ms):
    return [{"candidates": 1000, "pairs": 5000, "claim_ms": 0.0, "pair_ms": pair_ms}] * 2


def test_saturation_roofline_is_the_issue_roofline_of_the_pass_kernel():
    e = bench.load_profile("sq_issue.json", "php-res_B1")
    assert e, "profiles/sq_issue.json lacks the php-res entry"
    r = bench.saturation_roofline(_res_stats(0.25), nvars=12)
    assert r["kernel"].startswith("res_pass_packed_kernel")
    issue = bench.issue_roofline("php-res", 1, 0.25, kernel="res")
    for k in ("bound", "achieved", "peak", "frac", "unit"):
        assert r[k] == issue[k], k
    # the pipe fraction is the profiled instruction count over this run's time
    cyc = bench.PEAK_CLOCK_HZ * 0.25e-3
    peaks = {"valu": 1024 * 0.5 * cyc, "salu": 256 * cyc, "lds": 256 * cyc}
    counts = {"valu": e["valu_insts"], "salu": e["salu_insts"], "lds": e["lds_array_cycles"]}
    assert abs(r["frac"] - counts[r["bound"]] / peaks[r["bound"]]) < 1e-12
    assert r["kernel_ms_per_step"] == 0.25
    assert r["pairs_per_step"] == 5000 and r["candidates_per_step"] == 1000
    assert r["hbm_bytes_per_step"] == e.get("hbm_bytes_corrected")
    assert bench.saturation_roofline([], nvars=12) is None


def test_dp_roofline_prices_the_launch_chain():
    st = [{"launches": 280, "device_ms": 3.0, "subset_tests": 10, "new_clauses": 4, "words": 2}] * 3
    r = bench.dp_roofline(st, solves_per_s=300.0, floor_us=2.0)
    assert r["bound"] == "launch-latency" and r["unit"] == "launches/s"
    assert r["achieved"] == 280 * 300.0
    assert r["peak"] == 1e6 / 2.0 and r["floor_us_per_launch"] == 2.0
    assert r["peak_source"].startswith("measured")
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    assert abs(r["us_per_launch"] - 3.0e3 / 280) < 1e-9
    assert bench.dp_roofline([], 1.0, 2.0) is None


def test_saturation_roofline_prices_the_pipes_at_the_live_clock():
    """The pass kernels measure their own shader clock (s_memtime over
    s_memrealtime, satmi_resolution_last_clock): the roofline's pipe peaks
    are priced at the median live clock of the timed calls, with the
    peak-clock fractions beside it."""
    st = [dict(s, shader_clock_hz=hz) for s, hz in zip(_res_stats(0.25) * 2, (1.2e9, 1.4e9, 1.3e9, 1.3e9))]
    r = bench.saturation_roofline(st, nvars=12)
    assert r["clock_hz"] == 1.3e9 and r["clock_source"].startswith("live")
    peak = bench.saturation_roofline(_res_stats(0.25), nvars=12)
    assert peak["clock_source"] == "peak" and peak["clock_hz"] == bench.PEAK_CLOCK_HZ
    for k, v in r["fracs"].items():
        assert abs(v * 1.3e9 / bench.PEAK_CLOCK_HZ - peak["fracs"][k]) < 1e-12
        assert abs(r["fracs_at_peak_clock"][k] - peak["fracs"][k]) < 1e-12


def test_issue_roofline_staleness_follows_the_machine_code(monkeypatch):
    """`stale` compares the entry's kernel_isa_sha16 with the machine code of
    the kernel in the loaded library (satmi/isa.py), not the source text."""
    e = bench.load_profile("sq_issue.json", "php-res_B1")
    monkeypatch.setattr(bench, "kernel_isa_sha", lambda base: e["kernel_isa_sha16"])
    assert bench.issue_roofline("php-res", 1, 0.25, kernel="res")["stale"] is False
    monkeypatch.setattr(bench, "kernel_isa_sha", lambda base: "0" * 16)
    assert bench.issue_roofline("php-res", 1, 0.25, kernel="res")["stale"] is True


def test_every_profiled_kernel_is_found_in_the_library():
    import json
    import os
    import pytest
    from satmi import _capi, isa
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libsatmi.so not built")
    with open(os.path.join(os.path.dirname(bench.__file__), "profiles", "sq_issue.json")) as fh:
        table = json.load(fh)
    for key, e in table.items():
        sha = isa.kernel_code_sha(e["kernel"].split("<")[0])
        assert sha is not None and len(sha) == 16, key
        assert e.get("kernel_isa_sha16") and len(e["kernel_isa_sha16"]) == 16, key
