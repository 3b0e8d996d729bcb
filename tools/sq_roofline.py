"""Issue-pipe roofline inputs of the DPLL kernel from the SQ counter passes of
tools/profile_sq.sh, stored in profiles/sq_issue.json for bench.py.

    python tools/sq_roofline.py gpurun_out/<tag> [profiles/r02/<dir>]

Per launch of the bench workload (configs[2] unless the profiled bench line
says otherwise) it records the wave-instruction counts per pipe (SQ_INSTS_*),
the LDS-array cycles (SQ_LDS_IDX_ACTIVE, bank-conflict share beside it) and the
effective shader clock (GRBM_GUI_ACTIVE / 8 XCDs / profiled kernel time,
MI355X_MICROARCH.md "DVFS give-back").  bench.py divides the counts by the
live kernel duration and by the pipe peaks:

    VALU  0.5 wave-instructions / cycle / SIMD  (wave64 on SIMD-32: 2 cycles)
    SALU  1 instruction / cycle / CU            (one scalar unit per CU)
    LDS   1 array cycle / cycle / CU            (SQ_LDS_IDX_ACTIVE counts array cycles)

The counts are a property of the kernel build and the inputs (seeded), so the
entry carries the hash of the kernel source it was measured on; bench.py marks
the object stale when dpll_scan.hip has changed since.
"""
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL_SRC = os.path.join(ROOT, "sat-mpi-stana-andrei_amd", "csrc", "dpll_scan.hip")
OUT = os.path.join(ROOT, "profiles", "sq_issue.json")
CUS, SIMDS, XCDS = 256, 1024, 8


def kernel_hash():
    with open(KERNEL_SRC, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def read_summary(path):
    vals = {}
    with open(path) as fh:
        for line in fh:
            parts = line.split()
            if len(parts) >= 2:
                vals.setdefault(parts[0], float(parts[1]))   # GRBM_GUI_ACTIVE appears in both passes: keep pass 1
    return vals


def main():
    src = sys.argv[1]
    keep = sys.argv[2] if len(sys.argv) > 2 else None
    c = read_summary(os.path.join(src, "sq_summary.txt"))
    with open(os.path.join(src, "sq1.json")) as fh:
        bench = json.loads(fh.read().strip().splitlines()[-1])
    kms = bench["roofline"]["kernel_ms"]
    clock = c["GRBM_GUI_ACTIVE"] / XCDS / (kms * 1e-3)
    cyc = clock * kms * 1e-3
    workload = bench["config"]["preset"] + f"_B{bench['config']['instances_per_gpu']}"
    entry = {
        "kernel_src_sha256_16": kernel_hash(),
        "profiled_kernel_ms": kms,
        "effective_clock_hz": clock,
        "valu_insts": c["SQ_INSTS_VALU"], "salu_insts": c["SQ_INSTS_SALU"], "lds_insts": c["SQ_INSTS_LDS"],
        "branch_insts": c.get("SQ_INSTS_BRANCH"),
        "lds_array_cycles": c["SQ_LDS_IDX_ACTIVE"], "lds_bank_conflict_cycles": c["SQ_LDS_BANK_CONFLICT"],
        "wave_cycles_quad": c["SQ_WAVE_CYCLES"], "wait_any_quad": c.get("SQ_WAIT_ANY"),
        "wait_inst_any_quad": c.get("SQ_WAIT_INST_ANY"), "active_inst_any_quad": c.get("SQ_ACTIVE_INST_ANY"),
        "frac_at_profile": {
            "valu": c["SQ_INSTS_VALU"] / (SIMDS * 0.5 * cyc),
            "salu": c["SQ_INSTS_SALU"] / (CUS * cyc),
            "lds": c["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc),
        },
        "source": keep or src,
        "kernel": bench.get("roofline", {}).get("kernel"),   # the launch's kernel as the bench line names it
    }
    try:
        with open(OUT) as fh:
            table = json.load(fh)
    except (OSError, ValueError):
        table = {}
    table[workload] = entry
    with open(OUT, "w") as fh:
        json.dump(table, fh, indent=1, sort_keys=True)
    if keep:
        os.makedirs(os.path.join(ROOT, keep), exist_ok=True)
        for name in ("sq_summary.txt", "sq1.json", "sq2.json"):
            if os.path.exists(os.path.join(src, name)):
                shutil.copy(os.path.join(src, name), os.path.join(ROOT, keep, name))
    print(json.dumps({workload: entry}, indent=1))


if __name__ == "__main__":
    main()
