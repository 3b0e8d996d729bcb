#!/usr/bin/env python3
"""Benchmark: batched DPLL on random 3-SAT n=100, alpha=4.26 (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload P]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step = one pass of the hot path (csrc/dpll_scan.hip, SOUND mode, stop at the
first model: the SAT/UNSAT decision) over one batch of synthetic uniform random
3-SAT instances already resident in HBM, followed by the RCCL all-reduce of the
step's verdict/counter totals.  Consecutive steps alternate between two HIP
streams (and two resident batches), so one batch's tail overlaps the next
batch's start; the timed region still brackets all K steps with barrier +
synchronize.  The batch is BASELINE.json configs[2]: 262,144 instances of
n=100, alpha=4.26 per step, sharded across the ranks with no data-path
collective (strong scaling: 262,144 / N instances per GPU).  The batch is
generated in chunks of CHUNK instances, chunk c from seed + c, and a rank
materialises only the chunks of its shard: every N solves the same instances,
and the line's `verdict_sha` (the per-instance verdicts of the last step,
gathered over RCCL) is the same for every N.

--workload selects the other BASELINE.json configs (the default line is
configs[2]; at N = 1 the default run also measures every other config in a
child process after the headline -- the line's `configs` object):
    3sat-n50   configs[1]: 4,096 instances of n=50, alpha=4.26
    uf250      configs[4]: uf250-1065 shape (random 3-SAT n=250, m=1065),
               node-capped search (--node-limit, default 20,000 calls/instance)
    5sat-n200  configs[4]: random 5-SAT n=200 at the 5-SAT threshold
               (alpha=21.117, m=4,223): long clauses, 4 waves per CU of LDS,
               node-capped search (--node-limit, default 20,000)
    5sat-n200-a12  configs[4]: random 5-SAT n=200 at alpha 12 (m=2,400), every
               search decided to the end (no node limit) -- instances/s
    php-dp     configs[3]: Davis-Putnam elimination of pigeonhole PHP(6,5)
               (30 variables, 81 clauses; every step's resolvents, tautology
               and subsumption filter on the GPU) -- solves/s
    php-res    configs[3]: resolution saturation of PHP(4,3) (pair kernel +
               hash dedup), its first 4 passes (171,392 derived clauses; the
               5th pass would resolve 1.5e10 pairs) -- derived clauses/s
    rand-res / rand-dp  configs[3]'s small random UNSAT sets: 16 random 3-SAT
               formulas (n=7, m=49 / n=16, m=96) saturated by resolution /
               eliminated by Davis-Putnam to the end -- formulas/s
    cdcl       the reference's CDCLSolver (REF.py:217-384) on 32,768 menu-sized
               formulas (generate_large_formula(80, 3, 15), REF.py:21-29, the
               shape of rezultat.txt:178-188), <= 10,000 iterations each --
               formulas/s
For the node-capped workloads the headline value is unit-props/s.

Prints ONE JSON line on rank 0.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sat-mpi-stana-andrei_amd"))

import torch  # noqa: E402  (before libsatmi: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

from satmi import _capi, cnf, isa  # noqa: E402
from satmi.shard import gather_verdicts, shard_range  # noqa: E402

METRIC = "instances solved/sec, random 3-SAT n=100 α=4.26; unit-props/sec; HBM GB/s"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_CLOCK_HZ = 2.4e9          # MI355X peak engine clock (MI355X_MICROARCH.md: "2.4 GHz" issue rates)
SHADER_CLOCK_HZ = 2.4e9        # MI355X_MICROARCH.md: peak engine clock (the LDS-issue peak of dp_roofline)
CHUNK = 4096                   # instances per generation chunk (chunk c drawn from seed + c)
FIX_NCAP, FIX_MCAP = 127, 448  # dpll_fixed_kernel's shape class (csrc/dpll_scan.hip)

# workload presets: (total instances per step, n, alpha, k, node_limit, BASELINE config)
WORKLOADS = {
    "3sat-n100": (262144, 100, 4.26, 3, 0, "configs[2]"),
    "3sat-n50": (4096, 50, 4.26, 3, 0, "configs[1]"),
    "uf250": (8192, 250, 4.26, 3, 20000, "configs[4]"),        # 2 x the 4,096 resident waves (16 / CU)
    "5sat-n200": (2048, 200, 21.117, 5, 20000, "configs[4]"),  # 2 x the 1,024 resident waves (4 / CU)
    # configs[4]'s 5-SAT n=200 decided to the end: alpha 12 (m=2,400), where
    # every search of a batch finishes (at the threshold none of 64 did in 90 s:
    # profiles/r06/fullsolve_5sat_probe.txt)
    "5sat-n200-a12": (2048, 200, 12.0, 5, 0, "configs[4]"),
}
# configs[3] presets: (holes, resolution passes) -- one formula per step, host-array C ABI
SATURATION = {"php-dp": (5, 0), "php-res": (3, 4)}
# configs[3]'s "small random UNSAT sets": (solver, formulas per step, n, m, seed) --
# random 3-SAT past the threshold, each formula saturated / eliminated to the end
RANDSETS = {"rand-res": ("res", 16, 7, 49, 7001), "rand-dp": ("dp", 16, 16, 96, 7002)}
# CDCL preset: (formulas per step, clauses, max literals per clause, variables, max_iter, seed)
CDCL = {"cdcl": (32768, 80, 3, 15, 10000, 1234)}

# the secondary legs of the default N = 1 line: (name, workload, extra args)
LEGS = [
    ("configs[1] 2 streams", "3sat-n50", ["--streams", "2", "--steps", "32", "--warmup", "4"]),
    ("configs[1] 16 streams", "3sat-n50", ["--streams", "16", "--steps", "128", "--warmup", "16"]),
    ("configs[3] php-dp", "php-dp", ["--steps", "40", "--warmup", "3"]),
    ("configs[3] php-dp 8 threads", "php-dp", ["--steps", "10", "--warmup", "2", "--threads", "8"]),
    ("configs[3] php-res", "php-res", ["--steps", "20", "--warmup", "2"]),
    ("configs[3] rand-res", "rand-res", ["--steps", "3", "--warmup", "1"]),
    ("configs[3] rand-dp 8 threads", "rand-dp", ["--steps", "3", "--warmup", "1", "--threads", "8"]),
    ("configs[4] uf250", "uf250", ["--steps", "4", "--warmup", "1"]),
    ("configs[4] 5sat-n200", "5sat-n200", ["--steps", "4", "--warmup", "1"]),
    # configs[4] solved to the end (no node limit): 1,024 uf250-shaped searches per
    # step, branch splitting on with helper waves on every free CU slot (r06
    # sweep, profiles/r06/solved_sweep.txt: 512 per step 50.4-51.2/s at 10-24
    # helpers per CU, 1,024 per step 54.9/s at 16)
    ("configs[4] uf250 solved", "uf250", ["--node-limit", "0", "--total", "1024", "--split-always",
                                          "--helpers-per-cu", "16", "--steps", "2", "--warmup", "0",
                                          "--cpu-scaled"]),
    # 5-SAT n=200 decided to the end (alpha 12), split always: a step's time is
    # its hardest search's, so the batch is large (2,048 per step 172/s, 8,192
    # 354/s, 16,384 565/s: profiles/r06/solved_sweep.txt), two steps so that
    # one stream's tail overlaps the other's bulk (one step: 347/s)
    ("configs[4] 5sat-n200 solved", "5sat-n200-a12", ["--total", "16384", "--split-always", "--steps", "2",
                                                     "--warmup", "0", "--cpu-scaled"]),
    ("cdcl", "cdcl", ["--steps", "3", "--warmup", "1"]),
    ("cdcl 4 threads", "cdcl", ["--steps", "3", "--warmup", "1", "--threads", "4"]),
]
# legs run by a second child with a hardware queue per stream (GPU_MAX_HW_QUEUES,
# read at HIP start); the others keep HIP's default of 4 queues -- more queues
# cost concurrent host threads (php-dp with 8 threads: 1.09 k solves/s with 4
# queues, 0.71 k with 17; tools/hwq_sweep.sh)
HWQ17_LEGS = ("configs[1] 16 streams",)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", choices=sorted(WORKLOADS) + sorted(SATURATION) + sorted(RANDSETS) + sorted(CDCL),
                   default="3sat-n100")
    p.add_argument("--total", type=int, default=None, help="instances per step, all ranks")
    p.add_argument("--n", type=int, default=None)
    p.add_argument("--alpha", type=float, default=None)
    p.add_argument("--k", type=int, default=None)
    p.add_argument("--node-limit", type=int, default=None, help="dpll calls per instance (0 = none)")
    p.add_argument("--seed", type=int, default=20251016)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-scaled", action="store_true",
                   help="searches too long for any bounded CPU sample (uf250 solved to the end): the CPU sample is "
                        "node-capped at --cpu-sample-node-limit and its unit-props/s scaled to instances/s by the "
                        "GPU's unit propagations per instance (default: the oracle solves whole instances)")
    p.add_argument("--cpu-sample-node-limit", type=int, default=2000,
                   help="--cpu-scaled: the CPU sample's node cap")
    p.add_argument("--emulate-world", type=int, default=0,
                   help="on one GPU, run exactly rank --emulate-rank's shard of an N-rank job (the 8-GPU imbalance)")
    p.add_argument("--emulate-rank", type=int, default=0)
    p.add_argument("--full-json", default=None,
                   help="also write the uncompacted line (every leg's full objects) to this file")
    p.add_argument("--no-legs", action="store_true", help="only the headline workload (no `configs` object)")
    p.add_argument("--legs-only", action="store_true", help=argparse.SUPPRESS)   # the child of the default run
    p.add_argument("--legs-hwq17", action="store_true", help=argparse.SUPPRESS)  # ... its HWQ17_LEGS child
    p.add_argument("--leg-cpu-seconds", type=float, default=4.0, help="CPU baseline budget of each leg")
    p.add_argument("--profile-steps", action="store_true", help="no warmup/cpu leg (for rocprofv3 runs)")
    p.add_argument("--kernel", choices=("auto", "inc", "scan", "general"), default="auto",
                   help="DPLL kernel policy (satmi_dpll_set_kernel); auto = incremental clause kernel")
    p.add_argument("--no-split", action="store_true", help="disable branch splitting (satmi_dpll_set_split)")
    p.add_argument("--split-always", action="store_true",
                   help="split every eligible launch (default: at least 1 and at most 8 instances per resident wave)")
    p.add_argument("--split-warmup", type=int, default=-1,
                   help="nodes before a search may donate (satmi_dpll_set_split_warmup; -1 = default)")
    p.add_argument("--helpers-per-cu", type=int, default=0, help="branch-splitting helpers per CU (0 = library default)")
    p.add_argument("--threads", type=int, default=1,
                   help="php-dp / cdcl: concurrent solve calls per step, one host thread (and HIP stream) each")
    p.add_argument("--streams", type=int, default=None, choices=range(1, 17),
                   help="HIP streams (each with its own resident batch) the steps rotate over (default: 16 for "
                        "3sat-n50, whose 4,096 short searches leave most CU slots idle for a launch's 2 ms, else 2)")
    a = p.parse_args(argv)
    if a.workload in WORKLOADS:
        total, n, alpha, k, node_limit, a.config_name = WORKLOADS[a.workload]
        a.total = total if a.total is None else a.total
        a.n = n if a.n is None else a.n
        a.alpha = alpha if a.alpha is None else a.alpha
        a.k = k if a.k is None else a.k
        a.node_limit = node_limit if a.node_limit is None else a.node_limit
    return a


def init_ranks():
    """One process per GPU (torchrun env): (world, rank, local device).  The
    collective backend is RCCL ("nccl"); SATMI_DIST_BACKEND=gloo rehearses the
    multi-rank path with several ranks on fewer GPUs (device = LOCAL_RANK mod
    the visible GPUs) -- identical to the default on one rank per GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    if world > 1 and not dist.is_initialized():
        torch.cuda.set_device(local)
        backend = os.environ.get("SATMI_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def host_cores():
    """CPU cores this job may use: the box's share (OMP_NUM_THREADS is set to it
    on the GPU box; os.cpu_count() there shows the whole machine), else the
    affinity mask."""
    env = os.environ.get("SATMI_CPU_CORES") or os.environ.get("OMP_NUM_THREADS")
    return max(1, int(env) if env else len(os.sched_getaffinity(0)))


def cpu_pool(kind, icb, clb, lits, seconds, param):
    """oracle/cpu_pool.py as a child process (never touches the GPU), one worker
    per host core, on the CSR sample given."""
    import numpy as np
    cores = host_cores()
    with tempfile.TemporaryDirectory(prefix="satmi_cpu_") as tmp:
        for name, arr in (("icb", icb), ("clb", clb), ("lits", lits)):
            np.save(os.path.join(tmp, name + ".npy"), np.ascontiguousarray(arr, dtype=np.int32))
        env = {k: v for k, v in os.environ.items() if not k.startswith(("HIP_", "ROCR_", "HSA_", "GPU_"))}
        out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_pool.py"), kind, tmp, str(seconds),
                              str(param), str(cores)], check=True, capture_output=True, text=True, env=env)
    return json.loads(out.stdout.strip().splitlines()[-1]), cores


def cpu_baseline(batch_host, seconds, node_limit, props_per_instance=None, sample_node_limit=0):
    """The CPU oracle (oracle/, a C restatement of REF.py's DPLL, SOUND mode) on
    rank 0's host, on the same bench batch: one core (instances from the start
    of the batch until `seconds` / 3 pass), then every core (oracle/cpu_pool.py,
    one worker per core, for `seconds`).  `value` is the all-cores rate; the
    one-core rate is beside it.

    Searches solved to the end (node_limit 0) with sample_node_limit > 0: one
    uf250-shaped search is ~10^3 s of one host core (the oracle runs ~6 k
    nodes/s there), so no bounded sample finishes one.  The sample is then the
    same instances node-capped at sample_node_limit, and its unit-props/s is
    scaled to instances/s by the unit propagations per instance of the GPU's
    full solves of the same batch (bit-exact counters: the same searches)."""
    if node_limit == 0 and sample_node_limit > 0 and props_per_instance:
        r = cpu_baseline(batch_host, seconds, sample_node_limit)
        ups = r["unit_props_per_s"]
        r["sample_capped_instances_per_s"] = r.pop("instances_per_s")
        r.update({"value": ups / props_per_instance, "unit": "instances/s", "scaled_from": "unit-props/s",
                  "props_per_instance": props_per_instance,
                  "sample": r["sample"] + f"; scaled to instances/s by {props_per_instance:.4g} unit propagations "
                            f"per instance solved to the end (the GPU's counters on this batch)"})
        return r
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.lib()
    t0 = time.perf_counter()
    done = 0
    props = 0
    while done < batch_host.num_instances:
        r = oracle.dpll(batch_host.instance(done), "sound", max_solutions=1, sol_cap=1, node_limit=node_limit)
        props += r["counters"]["unit_props"]
        done += 1
        if time.perf_counter() - t0 > seconds / 3:
            break
    dt = time.perf_counter() - t0
    capped = node_limit > 0
    one = {"instances_per_s": done / dt, "unit_props_per_s": props / dt, "instances": done, "seconds": dt}
    cores = host_cores()
    # bounded sample for the pool: enough instances for every core for `seconds`
    nsamp = min(batch_host.num_instances, max(4 * cores, int(4 * cores * seconds * max(done, 1) / dt)))
    icb = batch_host.inst_clause_begin[:nsamp + 1].astype(np.int32)
    clb = batch_host.clause_lit_begin[:int(icb[-1]) + 1].astype(np.int32)
    lits = batch_host.lits[:int(clb[-1])].astype(np.int32)
    pool, cores = cpu_pool("dpll", icb, clb, lits, seconds, node_limit)
    rate = pool["unit_props_per_s"] if capped else pool["instances_per_s"]
    return {"value": rate, "unit": "unit-props/s" if capped else "instances/s",
            "cores": cores, "kind": "port",
            "sample": f"{pool['instances']} instances from the start of the rank-0 bench batch (same n/alpha"
                      f"{', node limit %d' % node_limit if capped else ''}), oracle/sat_oracle.c SOUND mode, "
                      f"{cores} worker processes (one per host core) for {pool['seconds']:.1f} s",
            "instances_per_s": pool["instances_per_s"], "unit_props_per_s": pool["unit_props_per_s"],
            "single_core": one}


def load_profile(name, key):
    try:
        with open(os.path.join(ROOT, "profiles", name)) as fh:
            return json.load(fh).get(key)
    except (OSError, ValueError):
        return None


def kernel_isa_sha(base):
    """16 hex digits of the machine code of the kernels named `base` in the
    loaded libsatmi.so (satmi/isa.py): the identity an SQ profile entry is
    keyed on, so a comment-only source edit does not make it stale."""
    return isa.kernel_code_sha(base)


def issue_roofline(preset, per_gpu, kernel_ms, kernel="dpll", clock_hz=None):
    """The DPLL kernel's binding resource is inside the CU: issue-pipe fractions
    from the SQ counter passes kept in profiles/sq_issue.json (tools/sq_roofline.py:
    wave-instructions / LDS-array cycles per launch of this exact workload) over
    this run's live kernel time at the peak engine clock.  Peaks: VALU 0.5
    wave-instructions / cycle / SIMD, SALU 1 / cycle / CU, LDS array 1 cycle /
    cycle / CU.  `stale` if the kernel's machine code in the loaded library differs from
    the code the profile was taken on (entry `kernel_isa_sha16`)."""
    e = load_profile("sq_issue.json", f"{preset}_B{per_gpu}")
    if not e:
        return None
    # the pipes' peak at the chip's peak engine clock (a short profiled kernel's
    # GRBM_GUI_ACTIVE-derived clock is not its live clock; a long one's, e.g.
    # the headline kernel's 2.39 GHz, is within 1 % of the peak), or at the
    # live clock the kernel measured itself (clock_hz: s_memtime over
    # s_memrealtime inside the kernel), with the peak-clock fractions beside it
    hz = clock_hz or PEAK_CLOCK_HZ
    cyc = hz * kernel_ms * 1e-3
    pipes = {"valu": (e["valu_insts"], 1024 * 0.5 * cyc, "wave-instr"),
             "salu": (e["salu_insts"], 256 * cyc, "instr"),
             "lds": (e["lds_array_cycles"], 256 * cyc, "array-cycles")}
    fr = {k: a / p for k, (a, p, _) in pipes.items()}
    bound = max(fr, key=fr.get)
    a, p, unit = pipes[bound]
    return {"bound": bound, "achieved": a / (kernel_ms * 1e-3), "peak": p / (kernel_ms * 1e-3),
            "unit": unit + "/s", "frac": fr[bound], "fracs": fr,
            "fracs_at_peak_clock": {k: v * hz / PEAK_CLOCK_HZ for k, v in fr.items()},
            "lds_bank_conflict_share": e["lds_bank_conflict_cycles"] / e["lds_array_cycles"],
            "clock_hz": hz, "clock_source": "live (in-kernel s_memtime / s_memrealtime)" if clock_hz else "peak",
            "profile_clock_hz": e["effective_clock_hz"], "source": e["source"],
            "kernel": e.get("kernel"),
            "stale": e.get("kernel_isa_sha16") != kernel_isa_sha(e.get("isa_symbol") or e["kernel"].split("<")[0])}


def dpll_kernel_name(n, m, k, split):
    """The kernel satmi_dpll_batch_device launches for this shape (csrc/dpll_scan.hip
    scan_plan / dpll_scan_launch; `split` = the launch used the splitting form)."""
    kern, _, _ = _capi.plan(n, m, m * k, k)
    if kern == _capi.KERNEL_INC and k == 3 and n <= FIX_NCAP and m <= FIX_MCAP:
        return f"dpll_fixed_kernel<{FIX_MCAP}, {'true' if split else 'false'}>"
    return {_capi.KERNEL_SCAN: "dpll_scan_kernel (full scans)", _capi.KERNEL_INC: "dpll_scan_kernel (incremental rounds)",
            _capi.KERNEL_GENERAL: "dpll_batch_kernel"}.get(kern, f"kernel {kern}")


def span_union_ms(spans, hz):
    """Length of the union of [begin, end) launch intervals (device ticks) in ms."""
    iv = sorted(spans)
    tot, cur_b, cur_e = 0, None, None
    for b, e in iv:
        if cur_e is None or b > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_b
            cur_b, cur_e = b, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_b
    return tot / hz * 1e3


def chunked_batch(b0, b1, n, m, k, seed, device):
    """Instances [b0, b1) of the virtual batch whose chunk c (instances
    [c*CHUNK, (c+1)*CHUNK)) is cnf.uniform_ksat_device(CHUNK, ..., seed + c):
    only the chunks overlapping [b0, b1) are drawn, so a rank's shard equals
    the same slice of the whole batch for every rank count."""
    B = b1 - b0
    if B <= 0:
        raise ValueError("empty shard")
    c0, c1 = b0 // CHUNK, (b1 - 1) // CHUNK + 1
    parts = []
    for c in range(c0, c1):
        _, _, lits, _ = cnf.uniform_ksat_device(CHUNK, n, m, k, seed=seed + c, device=device)
        lo = max(b0, c * CHUNK) - c * CHUNK
        hi = min(b1, (c + 1) * CHUNK) - c * CHUNK
        parts.append(lits.view(CHUNK, m * k)[lo:hi])
    lits = torch.cat(parts).reshape(-1).contiguous()
    icb = (torch.arange(B + 1, device=device, dtype=torch.int64) * m).to(torch.int32)
    clb = (torch.arange(B * m + 1, device=device, dtype=torch.int64) * k).to(torch.int32)
    nv = torch.full((B,), n, device=device, dtype=torch.int32)
    return icb, clb, lits, nv


def batch_seed(seed, j):
    """Seed base of resident batch j (one per stream), the same for every rank count."""
    return seed + 7919 * j


def run_dpll(args, world, rank, local):
    """One DPLL bench run (headline or leg): returns (line dict, host batch of the
    last step for the CPU baseline or None)."""
    NS = args.streams or (16 if args.workload == "3sat-n50" else 2)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    L = _capi.load()
    _capi.set_kernel({"auto": _capi.KERNEL_AUTO, "inc": _capi.KERNEL_INC, "scan": _capi.KERNEL_SCAN,
                      "general": _capi.KERNEL_GENERAL}[args.kernel])
    _capi.set_split(_capi.SPLIT_OFF if args.no_split else _capi.SPLIT_ALWAYS if args.split_always
                    else _capi.SPLIT_AUTO, args.helpers_per_cu)
    _capi.set_split_warmup(args.split_warmup)

    n, k = args.n, args.k
    # this rank's contiguous shard of the step's batch (--emulate-world: the
    # shard rank r of an N-rank job would get, run alone on this GPU)
    sw, sr = (args.emulate_world, args.emulate_rank) if args.emulate_world else (world, rank)
    b0, b1 = shard_range(args.total, sw, sr)
    B = b1 - b0
    m = int(round(args.alpha * n))
    # NS distinct resident batches, rotated step to step (batch j: the virtual
    # batch of seed base batch_seed(seed, j), this rank's slice of it)
    batches = [chunked_batch(b0, b1, n, m, k, batch_seed(args.seed, j), dev) for j in range(NS)]
    # NS streams, each with its own batch and output buffers: step j runs on
    # stream j % NS, so the next batch's waves take the CU slots that the
    # current batch's tail (its longest searches) leaves idle.  Launches on one
    # stream stay ordered, so a stream's buffers are reused only after its
    # previous step (kernel + verdict reduction) has finished.
    streams = [torch.cuda.Stream(dev) for _ in range(NS)]   # non-blocking pool streams
    outs = []
    for _ in range(NS):
        outs.append((torch.zeros(B, dtype=torch.int32, device=dev),
                     torch.zeros((B, _capi.NCOUNTERS), dtype=torch.int64, device=dev),
                     torch.zeros(B, dtype=torch.int32, device=dev),
                     torch.zeros((B, n), dtype=torch.int32, device=dev)))
    b_count = torch.tensor(B, device=dev, dtype=torch.int64)   # made once: a host->device copy per step would block
    spans = torch.zeros((max(args.steps, 1), 2), dtype=torch.int64, device=dev)

    def step(j, evs=None):
        s = streams[j % NS]
        icb, clb, lits, nv = batches[j % NS]
        status, counters, sol_len, sol_lits = outs[j % NS]
        with torch.cuda.stream(s):
            if evs is not None:
                evs[0].record(s)
            rc = L.satmi_dpll_batch_device(
                B, icb.data_ptr(), clb.data_ptr(), lits.data_ptr(), nv.data_ptr(), n, m, m * k, k, None, None,
                _capi.MODE_SOUND, 1, args.node_limit, 0.0, 1, n, status.data_ptr(), counters.data_ptr(),
                sol_len.data_ptr(), sol_lits.data_ptr(), None, None, s.cuda_stream)
            _capi.check(rc, "satmi_dpll_batch_device")
            if evs is not None:
                evs[1].record(s)
                # the kernel's own first-wave-start / last-wave-end clocks (overlap-proof)
                _capi.check(L.satmi_dpll_launch_span(s.cuda_stream, spans[j].data_ptr()), "satmi_dpll_launch_span")
            agg = torch.stack([(counters[:, 5] > 0).sum(), counters[:, 2].sum(), counters[:, 0].sum(),
                               (status > 2).sum() + (status == 2).sum() * (args.node_limit == 0),
                               (sol_len.to(torch.int64) * 4 + 4 * (counters[:, 5] > 0)).sum(),
                               counters[:, 7].sum(), b_count])
            if world > 1:
                dist.all_reduce(agg)   # RCCL: gather verdict/counter totals
        return agg

    def sync_all():
        for s in streams:
            s.synchronize()
        torch.cuda.synchronize()

    warm = 0 if args.profile_steps else args.warmup
    for j in range(warm):
        step(j)
    sync_all()
    if world > 1:
        dist.barrier()
    sync_all()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    aggs = [step(j, evs[j]) for j in range(args.steps)]
    sync_all()
    if world > 1:
        dist.barrier()
    sync_all()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    # launch duration of the DPLL kernel: its own clocks (first wave start to
    # last wave end, s_memrealtime), exact while the streams' launches overlap;
    # the HIP-event bracket on each stream is reported beside it (it also counts
    # the time a launch waits behind the other stream's tail).  The union of
    # the launch spans over the timed region is the time some launch ran: per
    # step it is <= ms_per_step (the overlap is what the streams buy).
    sp = spans.cpu().numpy().astype("uint64")
    hz = _capi.wallclock_hz()
    iv = [(int(~int(b) & (2**64 - 1)), int(e)) for b, e in sp[:args.steps]]
    span_ms = [(e - b) / hz * 1e3 for b, e in iv]
    kernel_ms = sum(span_ms) / len(span_ms)
    union_ms = span_union_ms(iv, hz)
    kms = [a.elapsed_time(b) for a, b in evs]
    event_ms = sum(kms) / len(kms)
    totals = torch.stack(aggs).sum(dim=0)
    last = (args.steps - 1) % NS
    status, counters, sol_len, sol_lits = outs[last]
    tot = totals.tolist()
    nsat, props, nodes, bad, written, ticks, all_inst = tot
    capped = args.node_limit > 0
    # node-capped workloads (configs[4]) measure search throughput: unit-props/s
    value = props / elapsed if capped else all_inst / elapsed

    # correctness check outside the timed region, on EVERY resident batch (the
    # last step of each stream): every reported model satisfies its formula
    def models_ok_for(j):
        icb_, clb_, lits_, nv_ = batches[j % NS]
        status_, counters_, sol_len_, sol_lits_ = outs[j % NS]
        sat_rows = counters_[:, 5] > 0
        val = torch.zeros((B, n + 1), dtype=torch.int8, device=dev)
        live = torch.arange(n, device=dev)[None, :] < sol_len_[:, None]
        idx = torch.where(live, sol_lits_.abs(), 0).to(torch.int64)
        val.scatter_(1, idx, torch.where(sol_lits_ > 0, 1, -1).to(torch.int8))
        val[:, 0] = 0
        lv = lits_.view(B, m, k).to(torch.int64)
        litval = torch.gather(val, 1, lv.abs().view(B, -1)).view(B, m, k) * torch.sign(lv).to(torch.int8)
        clause_ok = (litval > 0).any(dim=2).all(dim=1)
        return bool(((~sat_rows) | clause_ok).all().item())

    models_ok = all(models_ok_for(j) for j in range(max(0, args.steps - NS), args.steps))
    if not models_ok or bad:
        raise SystemExit(f"bench: invalid result (models_ok={models_ok}, limited={bad})")
    # the last step's per-instance verdicts gathered over the process group
    # (RCCL all-gather): the same hash for every rank count
    sat_last = (counters[:, 5] > 0).to(torch.int8)
    verdicts, ctr_tot = gather_verdicts(sat_last, counters, B if args.emulate_world else args.total, device=dev)
    seen = torch.ones(1, dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(seen)
    verdict_sha = hashlib.sha256(verdicts.cpu().numpy().tobytes()).hexdigest()[:16]
    icb, clb, lits, nv = batches[last]

    # roofline of the dominant kernel: algorithmic bytes per launch / average launch time
    read_bytes = B * (4 * m * k + 4 * m + 4 + 4) + 4
    write_bytes = B * (4 + 8 * _capi.NCOUNTERS) + written / all_inst * B
    alg_bytes = read_bytes + write_bytes
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    ach_excl = alg_bytes * args.steps / (union_ms * 1e-3) / 1e9
    workload = f"dpll_sound_{k}sat_n{n}_a{args.alpha}_B{B}"
    # resident waves of the persistent grid -> how busy the waves were (tail of the batch)
    kern, lds, per_cu = _capi.plan(n, m, m * k, k)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    st = _capi.split_stats(streams[last].cuda_stream) if not args.no_split else {"done": 0}
    split_used = bool(st["done"])
    # a splitting launch of a batch smaller than the CU slots adds helper waves
    # (csrc/dpll_scan.hip dpll_scan_launch): they count as resident
    extra = ncu * (args.helpers_per_cu or 1) if split_used else 0
    resident = min(B + extra, ncu * per_cu)
    # NS streams' launches overlap: at most every CU slot busy at once
    resident_all = min(NS * (B + extra), ncu * per_cu)
    # busy wave-time over resident wave-time of the timed region (all streams);
    # a splitting launch: each wave's own search time over the launch's waves x
    # its span, for the last launch of every stream (satmi_dpll_split_busy:
    # measured per wave, not through the rows a split search's helpers add to)
    util = ticks / world / hz / (resident_all * elapsed)
    if split_used:
        last_j = {j % NS: j for j in range(args.steps)}
        busy = sum(_capi.split_busy(streams[si].cuda_stream) for si in last_j)
        span_sum = sum(span_ms[j] for j in last_j.values()) * 1e-3
        util = busy / hz / (resident * span_sum) if span_sum > 0 else None
    pmc = load_profile("pmc_traffic.json", workload)
    kname = dpll_kernel_name(n, m, k, split_used)
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
            "kernel": kname, "kernel_ms": kernel_ms, "kernel_ms_hip_events": event_ms,
            "kernel_ms_exclusive": union_ms / args.steps, "achieved_exclusive": ach_excl,
            "frac_exclusive": ach_excl / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": alg_bytes,
            "overlap": f"{NS} streams: launches overlap, so kernel_ms (launch span, = rocprofv3's kernel "
                       f"duration) sums to {sum(span_ms) / args.steps:.1f} ms per step while some launch runs "
                       f"{union_ms / args.steps:.1f} ms per step (kernel_ms_exclusive <= ms_per_step)"}

    if capped:
        desc = (f"node-capped batched DPLL (SOUND mode, <= {args.node_limit} calls per instance), random {k}-SAT "
                f"n={n} alpha={args.alpha} m={m}, {args.total} instances per step sharded over {world} GPU(s) "
                f"(BASELINE {args.config_name})")
    else:
        desc = (f"batched DPLL (SOUND mode, first model = SAT/UNSAT decision), random {k}-SAT "
                f"n={n} alpha={args.alpha} m={m}, {args.total} instances per step sharded over "
                f"{world} GPU(s) (BASELINE {args.config_name})")
    out = {
        "metric": METRIC, "value": value, "unit": "unit-props/s" if capped else "instances/s", "n_gpus": world,
        "steps": args.steps, "warmup": warm, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int32",
        "data": f"synthetic: uniform random k-SAT generated in HBM (chunks of {CHUNK} seeded by chunk index: "
                f"the same instances for every N), {NS} batches rotated on {NS} streams",
        "config": {"workload": desc, "preset": args.workload, "node_limit": args.node_limit,
                   "instances_per_step": args.total, "instances_per_gpu": B, "n": n, "m": m, "k": k,
                   "parallelism": f"instance-sharded x{world}", "streams": NS,
                   "branch_splitting": not args.no_split,
                   "split_policy": "off" if args.no_split else "always" if args.split_always else "auto",
                   "helpers_per_cu": args.helpers_per_cu or 1, "split_warmup": args.split_warmup,
                   "emulated_shard": ({"world": sw, "rank": sr, "begin": b0, "end": b1} if args.emulate_world
                                      else None)},
        "instances_per_s": all_inst / elapsed,
        "unit_props_per_s": props / elapsed,
        "capped_fraction": int(((status == 2).sum()).item()) / B,
        "lds_bytes_per_wave": int(lds), "resident_waves": int(resident),
        "nodes_per_s": nodes / elapsed,
        "sat_fraction": nsat / all_inst,
        "hbm_gbs": achieved,
        "wave_utilisation": util,
        "verdict_sha": verdict_sha, "n_ranks_seen": int(seen.item()),
        "last_step_totals": {"sat": int((verdicts > 0).sum().item()), "nodes": int(ctr_tot[0].item()),
                             "unit_props": int(ctr_tot[2].item())},
        "roofline": roof,
        "roofline_issue": issue_roofline(args.workload, B, kernel_ms),
        "branch_split": st if split_used else None,   # None: the last launch did not split (auto policy)
    }
    host = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_steps:
        host = cnf.CnfBatch(icb.cpu().numpy(), clb.cpu().numpy(), lits.cpu().numpy(), nv.cpu().numpy())
    return out, host


def dp_roofline(stats, solves_per_s, floor_us):
    """Davis-Putnam (php-dp): a solve is a chain of dependent kernel launches
    (csrc/dp.hip: DP_LAUNCHES_PER_STEP per elimination step, 30 steps for
    PHP(6,5)) whose sizes live on the device, replayed from HIP graphs; most
    steps are small, so the chain's latency binds, not a pipe or HBM.
    achieved = launches completed per second; peak = the launch rate of an
    EMPTY dependent chain of the same length replayed from a HIP graph on this
    GPU, measured by the caller (`floor_us`, satmi_launch_chain_floor: one-block
    kernels, no work) -- the rate no chain of that many launches can beat;
    device_ms = the steps' device time (HIP events) per solve."""
    if not stats:
        return None
    launches = sum(s["launches"] for s in stats) / len(stats)
    dms = sum(s["device_ms"] for s in stats) / len(stats)
    ach = launches * solves_per_s
    peak = 1e6 / floor_us
    return {"bound": "launch-latency", "achieved": ach, "peak": peak, "unit": "launches/s", "frac": ach / peak,
            "peak_source": "measured: an empty chain of as many dependent one-block launches replayed from a HIP "
                           "graph (satmi_launch_chain_floor)", "floor_us_per_launch": floor_us,
            "traffic": None, "kernel": "dp step chain (8 kernels per elimination step)",
            "launches_per_solve": launches, "device_ms_per_solve": dms,
            "us_per_launch": dms * 1e3 / launches if launches else None,
            "subset_tests_per_solve": sum(s["subset_tests"] for s in stats) / len(stats),
            "new_clauses_per_solve": sum(s["new_clauses"] for s in stats) / len(stats), "key_words": stats[-1]["words"]}


def dp_launch_floor(stats):
    """satmi_launch_chain_floor over a chain as long as a solve's (after the timed region)."""
    if not stats:
        return None
    n = max(1, int(round(sum(s["launches"] for s in stats) / len(stats))))
    return _capi.launch_chain_floor(n, reps=20)


def saturation_roofline(stats, nvars):
    """Resolution (php-res, <= 31 variables): one fused pass kernel per
    saturation pass (csrc/resolution.hip res_pass_packed_kernel: pair
    classification + claims in a table that stays in L2/MALL), timed per step
    by HIP events.  Its binding pipe comes from the SQ passes of
    tools/pmc_workload.sh (profiles/sq_issue.json "php-res_B1", per step): the
    issue roofline over this run's live kernel time; the HBM bytes per step
    (FETCH x2 + WRITE, the same passes) beside it -- a small fraction of HBM:
    the table and the keys are cache-resident."""
    if not stats:
        return None
    pms = sum(s["pair_ms"] for s in stats) / len(stats)
    clocks = sorted(s["shader_clock_hz"] for s in stats if s.get("shader_clock_hz"))
    live_hz = clocks[len(clocks) // 2] if clocks else None   # median over the timed calls
    roof = issue_roofline("php-res", 1, pms, kernel="res", clock_hz=live_hz)
    if roof is None:
        return None
    e = load_profile("sq_issue.json", "php-res_B1") or {}
    roof.update({"kernel": "res_pass_packed_kernel (fused pairs + claims)", "kernel_ms_per_step": pms,
                 "pairs_per_step": sum(s["pairs"] for s in stats) / len(stats),
                 "candidates_per_step": sum(s["candidates"] for s in stats) / len(stats),
                 "hbm_bytes_per_step": e.get("hbm_bytes_corrected"),
                 "hbm_frac": (e["hbm_bytes_corrected"] / (pms * 1e-3) / 1e9 / HBM_PEAK_GBS)
                 if e.get("hbm_bytes_corrected") else None})
    return roof


def run_saturation(args, world, rank, local):
    """configs[3]: Davis-Putnam / resolution saturation of a pigeonhole formula.
    A step = one full satmi_dp_host / satmi_resolution_host call (host arrays in,
    verdict out: the boundary these solvers have, REF.py:63-130).  Each rank
    solves its own replica (one formula does not shard)."""
    from satmi.dp import eliminate
    from satmi.dp import last_stats as dp_stats
    from satmi.resolution import last_stats as res_stats
    from satmi.resolution import resolve
    from concurrent.futures import ThreadPoolExecutor
    torch.cuda.set_device(local)
    holes, npass = SATURATION[args.workload]
    f = cnf.pigeonhole(holes)
    T = max(1, args.threads) if args.workload == "php-dp" else 1
    if args.workload == "php-dp":
        def one():   # statistics are per host thread: read them in the thread that solved
            torch.cuda.set_device(local)
            r = eliminate(f)
            return r, dp_stats()
        work = lambda r: 1                                          # noqa: E731
        unit, metric_desc = "solves/s", f"Davis-Putnam elimination of PHP({holes + 1},{holes})"
    else:
        def one():
            r = resolve(f, max_passes=npass)
            return r, res_stats()
        work = lambda r: sum(r["pass_new"])                         # noqa: E731
        unit, metric_desc = "derived clauses/s", f"resolution saturation of PHP({holes + 1},{holes}), first {npass} passes"
    pool = ThreadPoolExecutor(T) if T > 1 else None
    # a step: T concurrent solves (one host thread and HIP stream each; T = 1: one solve)
    run = (lambda: list(pool.map(lambda _: one(), range(T)))) if pool else (lambda: [one()])   # noqa: E731
    for _ in range(0 if args.profile_steps else args.warmup):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    done = 0
    last = None
    stats = []
    for _ in range(args.steps):
        outs = run()
        for r, st in outs:
            done += work(r)
            stats.append(st)
        last = outs[-1][0]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=torch.device("cuda", local))
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    if pool:
        pool.shutdown()
    out = {"metric": METRIC, "value": done * world / elapsed, "unit": unit, "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic: pigeonhole formula",
           "config": {"workload": metric_desc + " (BASELINE configs[3]); replicas across ranks"
                                  + (f"; {T} concurrent solves per step (host threads, one HIP stream each)" if T > 1
                                     else ""),
                      "preset": args.workload, "parallelism": f"replicas x{world}", "concurrent_solves": T},
           "result": last["result"], "passes_or_steps": last.get("passes", last.get("steps")),
           "roofline": saturation_roofline(stats, len({abs(l) for c in f for l in c})) if args.workload == "php-res" else
           dp_roofline(stats, done * world / elapsed, dp_launch_floor(stats))}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_steps:
        # the oracle on the same formula: checked against the GPU, then replicas
        # on every host core (oracle/cpu_pool.py)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        r = oracle.dp(f) if args.workload == "php-dp" else oracle.resolution(f, max_passes=npass)
        # per pass (resolution: every pass's new-clause count) / per step (DP)
        per = (lambda x: [x["steps"], list(x["vars"])]) if args.workload == "php-dp" else (lambda x: list(x["pass_new"]))   # noqa: E731
        if r["result"] != last["result"] or per(r) != per(last):
            raise SystemExit(f"bench: GPU and oracle disagree on the configs[3] workload: "
                             f"{last['result']} {per(last)} vs {r['result']} {per(r)}")
        out["oracle_check"] = {"result": r["result"], ("steps_vars" if args.workload == "php-dp" else "pass_new"): per(r)}
        hb = cnf.pack([f])
        pool, cores = cpu_pool("dp" if args.workload == "php-dp" else "res", hb.inst_clause_begin,
                               hb.clause_lit_begin, hb.lits, args.cpu_seconds, npass)
        cpu = {"value": pool["units_per_s"], "unit": unit, "cores": cores, "kind": "port",
               "sample": f"{metric_desc} by the oracle (oracle/*.c) replicated on {cores} worker processes "
                         f"(one per host core) for {pool['seconds']:.1f} s: {pool['units']} units",
               "single_core_estimate": pool["units_per_s"] / cores}
    out["cpu_baseline"] = cpu
    return out


def run_cdcl(args, world, rank, local):
    """The reference's CDCLSolver (REF.py:217-384) batched on the GPU
    (csrc/cdcl.hip, one wavefront per formula): a step = one satmi_cdcl_batch_host
    call over the preset's formulas (host arrays in, verdicts out), each run to
    its verdict or max_iter iterations (the reference's own loop is unbounded;
    its driver times it out).  Replicas across ranks."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from satmi.cdcl import CDCL_LIMIT, CDCL_SAT, CDCL_UNSAT, STAT_NAMES, cdcl_batch_packed
    torch.cuda.set_device(local)
    nf, ncl, maxlit, nvar, max_iter, seed = CDCL[args.workload]
    T = max(1, args.threads)
    # the CSR host arrays the C ABI takes: one batch per concurrent solve
    # (seed + thread index), thread 0's is the one checked and CPU-timed
    hbs = [cnf.menu_batch(nf, ncl, maxlit, nvar, seed=seed + t) for t in range(T)]
    hb = hbs[0]
    pool_ex = ThreadPoolExecutor(T) if T > 1 else None

    from satmi.cdcl import last_stats as cdcl_stats

    def one(b):   # launch statistics are per host thread: read them in the thread that solved
        r = cdcl_batch_packed(b, max_iter=max_iter, arrays=True)
        r["launch"] = cdcl_stats()
        return r

    def step():
        if pool_ex is None:
            return [one(hb)]
        return list(pool_ex.map(one, hbs))

    for _ in range(0 if args.profile_steps else args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if pool_ex is not None:
        pool_ex.shutdown()
    launch = [r["launch"] for r in res]
    span_ms = sum(x["span_s"] for x in launch) / len(launch) * 1e3
    util = sum(x["busy_wave_s"] for x in launch) / sum(x["resident_waves"] * x["span_s"] for x in launch)
    el = torch.tensor([elapsed], dtype=torch.float64, device=torch.device("cuda", local))
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    st = np.concatenate([r["status"] for r in res])
    iters = int(sum(r["stats"][:, STAT_NAMES.index("iterations")].sum() for r in res))
    out = {"metric": METRIC, "value": nf * T * args.steps * world / elapsed, "unit": "formulas/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32/f64 activities",
           "data": f"synthetic: {nf} formulas of generate_large_formula({ncl}, {maxlit}, {nvar})'s distribution "
                   f"per solve call (REF.py:21-29; satmi.cnf.menu_batch, seed {seed}"
                   + (f"..{seed + T - 1}, one per concurrent call)" if T > 1 else ")"),
           "config": {"workload": f"cdcl_solve (REF.py:382-384) on {nf} formulas, <= {max_iter} iterations each; "
                                  f"replicas across ranks"
                                  + (f"; {T} concurrent calls per step (host threads, one HIP stream each)"
                                     if T > 1 else ""), "preset": args.workload,
                      "parallelism": f"replicas x{world}", "concurrent_solves": T},
           "sat": int((st == CDCL_SAT).sum()), "unsat": int((st == CDCL_UNSAT).sum()),
           "iteration_capped": int((st == CDCL_LIMIT).sum()),
           "iterations_per_s": iters * args.steps * world / elapsed,
           "kernel_ms": span_ms, "wave_utilisation": util,
           "roofline": issue_roofline(args.workload, nf, span_ms, kernel="cdcl")}
    r0 = res[0]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_steps:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        for i in range(0, nf, max(1, nf // 16)):   # verdicts checked against the oracle on a sample
            o = oracle.cdcl(hb.instance(i), max_iter=max_iter)
            g = {CDCL_SAT: 1, CDCL_UNSAT: 0, CDCL_LIMIT: -1}.get(int(r0["status"][i]), -2)
            if o["result"] != g or (g == 1 and o["assignment"] != r0["assign"][i, :r0["assign_len"][i]].tolist()):
                raise SystemExit(f"bench: GPU and oracle disagree on CDCL formula {i}")
        pool, cores = cpu_pool("cdcl", hb.inst_clause_begin, hb.clause_lit_begin, hb.lits, args.cpu_seconds,
                               max_iter)
        cpu = {"value": pool["units_per_s"], "unit": "formulas/s", "cores": cores, "kind": "port",
               "sample": f"{pool['units']} of the same formulas by oracle/cdcl_oracle.c on {cores} worker "
                         f"processes (one per host core) for {pool['seconds']:.1f} s"}
    out["cpu_baseline"] = cpu
    return out


def run_randset(args, world, rank, local):
    """configs[3]'s small random UNSAT sets: a step = every formula of a fixed
    set of random 3-SAT formulas past the threshold saturated by resolution
    (REF.py:63-95, to the empty clause or no new clause) or eliminated by
    Davis-Putnam (REF.py:98-130), one satmi call per formula (host arrays in,
    verdict out); `--threads` T splits the set over T host threads (one HIP
    stream each).  Each rank solves its own replica of the set."""
    from satmi.dp import eliminate
    from satmi.resolution import resolve
    from concurrent.futures import ThreadPoolExecutor
    torch.cuda.set_device(local)
    kind, count, n, m, seed = RANDSETS[args.workload]
    batch = cnf.uniform_ksat(count, n, m, 3, seed=seed)
    fs = [batch.instance(b) for b in range(count)]
    T = max(1, args.threads)

    def part(t):
        torch.cuda.set_device(local)
        return [(b, resolve(fs[b]) if kind == "res" else eliminate(fs[b])) for b in range(t, count, T)]

    pool = ThreadPoolExecutor(T) if T > 1 else None
    run = (lambda: sorted(x for ys in pool.map(part, range(T)) for x in ys)) if pool else (lambda: part(0))   # noqa: E731
    for _ in range(0 if args.profile_steps else args.warmup):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    derived = 0
    last = None
    for _ in range(args.steps):
        last = run()
        derived += sum(sum(r["pass_new"]) for _, r in last) if kind == "res" else 0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=torch.device("cuda", local))
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    if pool:
        pool.shutdown()
    results = [r["result"] for _, r in last]
    desc = (f"{'resolution saturation' if kind == 'res' else 'Davis-Putnam elimination'} of {count} random 3-SAT "
            f"formulas n={n} m={m} (alpha={m / n:g}) to the end")
    out = {"metric": METRIC, "value": count * args.steps * world / elapsed, "unit": "formulas/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
           "data": "synthetic: seeded uniform random 3-SAT",
           "config": {"workload": desc + " (BASELINE configs[3]: small random UNSAT sets); replicas across ranks"
                                  + (f"; {T} host threads" if T > 1 else ""),
                      "preset": args.workload, "parallelism": f"replicas x{world}", "concurrent_solves": T},
           "result": results, "unsat": results.count(0), "roofline": None}
    if kind == "res":
        out["derived_clauses_per_s"] = derived * world / elapsed
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_steps:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        # the oracle on the first formulas (resolution: ~2 s each on one core): verdicts
        # and per-pass counts / eliminated variables checked against the GPU's
        nchk = 2 if kind == "res" else count
        for b, r in last[:nchk]:
            o = oracle.resolution(fs[b]) if kind == "res" else oracle.dp(fs[b])
            got = (r["result"], list(r["pass_new"])) if kind == "res" else (r["result"], list(r["vars"]))
            exp = (o["result"], list(o["pass_new"])) if kind == "res" else (o["result"], list(o["vars"]))
            if got != exp:
                raise SystemExit(f"bench: GPU and oracle disagree on {args.workload} formula {b}: {got} vs {exp}")
        out["oracle_check"] = {"formulas_checked": nchk}
        pres, cores = cpu_pool(kind + "set", batch.inst_clause_begin, batch.clause_lit_begin, batch.lits,
                               args.cpu_seconds, 0)
        cpu = {"value": pres["units_per_s"], "unit": "formulas/s", "cores": cores, "kind": "port",
               "sample": f"the same {count} formulas by the oracle (oracle/*.c), worker w solving formulas w, "
                         f"w + {cores}, ... (cycling) on {cores} worker processes (one per host core) for "
                         f"{pres['seconds']:.1f} s: {pres['units']} formulas"}
    out["cpu_baseline"] = cpu
    return out


def run_one(args, world, rank, local):
    if args.workload in SATURATION:
        return run_saturation(args, world, rank, local)
    if args.workload in RANDSETS:
        return run_randset(args, world, rank, local)
    if args.workload in CDCL:
        return run_cdcl(args, world, rank, local)
    out, host = run_dpll(args, world, rank, local)
    ppi = out["unit_props_per_s"] / out["instances_per_s"] if out["instances_per_s"] else None
    scaled = args.cpu_sample_node_limit if args.cpu_scaled else 0
    out["cpu_baseline"] = (cpu_baseline(host, args.cpu_seconds, args.node_limit, ppi, scaled)
                           if host is not None else None)
    return out


def legs_main(args):
    """The default run's children: every other BASELINE config, short, one JSON
    object {name: compact line}.  Child processes so that the 16-stream leg
    gets a hardware queue per stream (GPU_MAX_HW_QUEUES, read at HIP start:
    --legs-hwq17 runs HWQ17_LEGS, the other child the rest)."""
    out = {}
    for name, wl, extra in LEGS:
        if (name in HWQ17_LEGS) != args.legs_hwq17:
            continue
        a = parse(["--workload", wl, "--cpu-seconds", str(args.leg_cpu_seconds), "--seed", str(args.seed)] + extra)
        t = time.perf_counter()
        r = run_one(a, 1, 0, 0)
        r["leg_wall_s"] = time.perf_counter() - t
        out[name] = r
        # progress on stderr (inherited by the parent: a long default run keeps
        # telling a watchdog it is alive; stdout carries only the result)
        print(f"bench: leg {name!r} done in {r['leg_wall_s']:.1f} s", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


# The printed line stays well inside what the driver parses (r05's 25 KB line
# was not parsed; r04's 17.5 KB was): the headline keeps its full roofline,
# issue roofline and CPU baseline, each leg only its figures.  --full-json
# writes the uncompacted line beside it.
LINE_BUDGET = 8000
HEAD_ROOF = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms", "kernel_ms_hip_events",
             "kernel_ms_exclusive", "frac_exclusive", "algorithmic_bytes_per_launch")
HEAD_ISSUE = ("bound", "achieved", "peak", "unit", "frac", "fracs", "lds_bank_conflict_share", "clock_source",
              "kernel", "source", "stale")
HEAD_CPU = ("value", "unit", "cores", "kind", "sample")
HEAD_DROP = ("configs", "configs_note", "branch_split", "roofline", "roofline_issue", "cpu_baseline")


def _sig(x, digits=4):
    """Floats to `digits` significant digits, recursively (the line's size)."""
    if isinstance(x, float):
        return float(f"{x:.{digits}g}")
    if isinstance(x, dict):
        return {k: _sig(v, digits) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_sig(v, digits) for v in x]
    return x


def _pick(d, keys):
    return {k: d[k] for k in keys if d and k in d} if d else None


def compact_leg(r):
    """A secondary config's figures: value, unit, time per step, the binding
    roofline fractions, the CPU baseline and the verdict hash."""
    out = {k: r[k] for k in ("value", "unit", "ms_per_step", "steps") if k in r}
    roof, iss, cpu = r.get("roofline"), r.get("roofline_issue"), r.get("cpu_baseline")
    out["roofline"] = _pick(roof, ("bound", "frac"))
    if iss:
        out["roofline_issue"] = _pick(iss, ("bound", "frac", "stale"))
    out["cpu_baseline"] = _pick(cpu, ("value", "unit", "cores"))
    for k in ("verdict_sha", "capped_fraction", "wave_utilisation"):
        if k in r:
            out[k] = r[k]
    return _sig(out)


def compact_line(full):
    """The printed line: every contract key and the headline's figures in full,
    its roofline / issue roofline / CPU baseline trimmed to their figures, the
    legs compacted (compact_leg)."""
    out = {k: v for k, v in full.items() if k not in HEAD_DROP}
    out["roofline"] = _sig(_pick(full.get("roofline"), HEAD_ROOF))
    if full.get("roofline_issue") is not None:
        out["roofline_issue"] = _sig(_pick(full["roofline_issue"], HEAD_ISSUE))
    cpu = full.get("cpu_baseline")
    if cpu is not None:
        c = _pick(cpu, HEAD_CPU)
        if isinstance(cpu.get("single_core"), dict):
            c["single_core_value"] = cpu["single_core"].get("instances_per_s")
        out["cpu_baseline"] = _sig(c)
    bs = full.get("branch_split")
    if bs:
        out["branch_split"] = dict(bs)
    if "configs" in full:
        out["configs"] = {name: compact_leg(r) for name, r in full["configs"].items()}
    return out


def main():
    args = parse()
    if args.legs_only:
        return legs_main(args)
    world, rank, local = init_ranks()
    if args.emulate_world and (world > 1 or not 0 <= args.emulate_rank < args.emulate_world):
        raise SystemExit("bench: --emulate-world runs one rank's shard in a 1-process job (0 <= rank < world)")
    if args.workload == "3sat-n50" and (args.streams or 16) > 3 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 17:
        print("bench: note: GPU_MAX_HW_QUEUES < streams + 1, the streams share hardware queues", file=sys.stderr)
    t_start = time.perf_counter()
    out = run_one(args, world, rank, local)
    if rank == 0:
        print(f"bench: {args.workload} done in {time.perf_counter() - t_start:.1f} s", file=sys.stderr, flush=True)
    legs = (world == 1 and not args.no_legs and not args.profile_steps and args.workload == "3sat-n100"
            and args.total == WORKLOADS["3sat-n100"][0] and not args.emulate_world)
    if legs and rank == 0:
        got = {}
        for hwq in (False, True):
            env = dict(os.environ, GPU_MAX_HW_QUEUES="17") if hwq else dict(os.environ)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--legs-only", "--seed", str(args.seed),
                                "--leg-cpu-seconds", str(args.leg_cpu_seconds)]
                               + (["--legs-hwq17"] if hwq else [])
                               + (["--no-cpu-baseline"] if args.no_cpu_baseline else []),
                               stdout=subprocess.PIPE, text=True, env=env)   # (stderr: the legs' progress)
            if r.returncode != 0:
                raise SystemExit(f"bench: secondary configs failed (exit {r.returncode}; their stderr above)")
            got.update(json.loads(r.stdout.strip().splitlines()[-1]))
        # (DESIGN.md "Measurement": how the legs run and which answers configs[1])
        out["configs"] = {name: got[name] for name, _, _ in LEGS if name in got}
    if rank == 0:
        out["wall_s"] = time.perf_counter() - t_start
        if args.full_json:
            with open(args.full_json, "w") as fh:
                json.dump(out, fh)
        print(json.dumps(compact_line(out)), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
