"""Issue-pipe roofline inputs of a kernel from tools/pmc_workload.sh's SQ passes
(sq1 + sq2), stored in profiles/sq_issue.json for bench.py's issue_roofline().

    python tools/sq_issue_entry.py gpurun_out/<tag> <workload> <kernel substring> <key> <src> [keep dir] [--per-step]
        [--isa-symbol=<mangled-name substring of the launched instance>]

--per-step: a step of the workload is several launches (resolution: one pass
kernel per saturation pass), so the counts are divided by the bench line's
steps + warmup instead of by the dispatches, and the live time is the line's
roofline.kernel_ms_per_step.

Per launch (the counters summed over the kernel's dispatches / dispatches):
wave-instructions per pipe (SQ_INSTS_*), LDS-array cycles (SQ_LDS_IDX_ACTIVE,
bank-conflict cycles beside it), and the effective clock = GRBM_GUI_ACTIVE per
XCD / the live launch time the profiled bench line reports (`kernel_ms`).
bench.py divides the counts by the live kernel time and the pipe peaks (VALU
0.5 wave-instr / cycle / SIMD, SALU 1 / cycle / CU, LDS 1 array cycle / cycle /
CU); the entry carries the kernel's machine-code hash (satmi/isa.py: stale when the
code object changes, not on comment edits) and, for reference, the source hash.
"""
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "sq_issue.json")
CUS, SIMDS, XCDS = 256, 1024, 8


def main():
    argv = [a for a in sys.argv[1:] if a != "--per-step" and not a.startswith("--isa-symbol=")]
    per_step = "--per-step" in sys.argv
    # the kernel instance the profiled workload launches (a mangled-name substring,
    # e.g. dpll_scan_kernelILi3ELi512ELb1ELb0E); default: every instance of kname
    isa_symbol = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--isa-symbol=")), None)
    src, wl, kname, key, ksrc = argv[:5]
    keep = argv[5] if len(argv) > 5 else None
    vals, ndisp = {}, {}
    section = None
    with open(os.path.join(src, f"pmc_{wl}.txt")) as fh:
        for line in fh:
            if line.startswith("=="):
                section = line.split("kernel", 1)[1].strip()
                continue
            parts = line.split()
            if section == kname and len(parts) >= 3:
                vals.setdefault(parts[0], float(parts[1]))
                ndisp.setdefault(parts[0], int(parts[2].split("=")[1]))
    nd = ndisp["SQ_INSTS_VALU"]
    with open(os.path.join(src, "p1.json")) as fh:
        bench = json.loads(fh.read().strip().splitlines()[-1])
    if per_step:
        kms = bench["roofline"]["kernel_ms_per_step"]
        nunits = bench["steps"] + bench["warmup"]
        per = lambda k: vals[k] / nunits   # noqa: E731
    else:
        kms = bench.get("kernel_ms") or bench["roofline"]["kernel_ms"]
        per = lambda k: vals[k] / ndisp[k]   # noqa: E731
    clock = per("GRBM_GUI_ACTIVE") / XCDS / (kms * 1e-3)
    cyc = clock * kms * 1e-3
    with open(os.path.join(ROOT, "sat-mpi-stana-andrei_amd", "csrc", ksrc), "rb") as fh:
        sha = hashlib.sha256(fh.read()).hexdigest()[:16]
    # the staleness key: the kernel's machine code in the in-tree libsatmi.so
    # (the library the profiled run shipped with -- enter the profile before
    # rebuilding)
    sys.path.insert(0, os.path.join(ROOT, "sat-mpi-stana-andrei_amd"))
    from satmi import isa
    isa_symbol = isa_symbol or kname.split("<")[0]
    isa_sha = isa.kernel_code_sha(isa_symbol)
    entry = {
        "kernel": kname, "kernel_src_sha256_16": sha, "kernel_isa_sha16": isa_sha, "isa_symbol": isa_symbol, "dispatches": nd, "profiled_kernel_ms": kms,
        "per": "step" if per_step else "launch",
        "effective_clock_hz": clock,
        "valu_insts": per("SQ_INSTS_VALU"), "salu_insts": per("SQ_INSTS_SALU"), "lds_insts": per("SQ_INSTS_LDS"),
        "branch_insts": per("SQ_INSTS_BRANCH"), "vmem_rd_insts": per("SQ_INSTS_VMEM_RD"),
        "lds_array_cycles": per("SQ_LDS_IDX_ACTIVE"), "lds_bank_conflict_cycles": per("SQ_LDS_BANK_CONFLICT"),
        "waves": per("SQ_WAVES"), "wave_cycles_quad": per("SQ_WAVE_CYCLES"), "busy_cycles": per("SQ_BUSY_CYCLES"),
        "wait_inst_any_quad": per("SQ_WAIT_INST_ANY"), "active_inst_any_quad": per("SQ_ACTIVE_INST_ANY"),
        "frac_at_profile": {
            "valu": per("SQ_INSTS_VALU") / (SIMDS * 0.5 * cyc),
            "salu": per("SQ_INSTS_SALU") / (CUS * cyc),
            "lds": per("SQ_LDS_IDX_ACTIVE") / (CUS * cyc),
        },
        "source": keep or src,
    }
    try:
        with open(OUT) as fh:
            table = json.load(fh)
    except (OSError, ValueError):
        table = {}
    table[key] = entry
    with open(OUT, "w") as fh:
        json.dump(table, fh, indent=1, sort_keys=True)
    if keep:
        os.makedirs(os.path.join(ROOT, keep), exist_ok=True)
        shutil.copy(os.path.join(src, f"pmc_{wl}.txt"), os.path.join(ROOT, keep, f"pmc_{wl}.txt"))
        shutil.copy(os.path.join(src, "p1.json"), os.path.join(ROOT, keep, f"pmc_{wl}_bench.json"))
    # HBM bytes from the FETCH_SIZE / WRITE_SIZE passes when present (KB units;
    # FETCH x2 per MI355X_MICROARCH.md's gfx950 correction, raw beside it)
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        entry["fetch_bytes_raw"] = per("FETCH_SIZE") * 1024
        entry["hbm_bytes_corrected"] = 2 * per("FETCH_SIZE") * 1024 + per("WRITE_SIZE") * 1024
        table[key] = entry
        with open(OUT, "w") as fh:
            json.dump(table, fh, indent=1, sort_keys=True)
    print(json.dumps({key: entry}, indent=1))


if __name__ == "__main__":
    main()
