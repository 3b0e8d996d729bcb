"""Diagnostic: one batched-DPLL launch, with per-instance tick accounting.

    python tools/dpll_probe.py [--per-gpu B] [--n 100] [--alpha 4.26] [--k 3] [--reps 2]

Prints kernel time (HIP events on the launch stream), the node/prop totals,
the wave utilisation (sum of per-instance wave ticks / (resident waves x kernel
time)) and the slowest instance -- the tail of the persistent grid.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sat-mpi-stana-andrei_amd"))
import torch  # noqa: E402
from satmi import _capi, cnf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-gpu", type=int, default=32768)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--alpha", type=float, default=4.26)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--lib", default=None, help="load this libsatmi build instead (experiments)")
    ap.add_argument("--kernel", choices=("auto", "general", "scan", "inc"), default="auto")
    ap.add_argument("--diag", action="store_true", help="load libsatmi_diag.so (or --lib, a diag build) and report per-phase clocks")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.lib:
        _capi.LIB_PATH = os.path.abspath(a.lib)
    if a.diag and not a.lib:
        _capi.LIB_PATH = os.path.join(os.path.dirname(_capi.LIB_PATH), "libsatmi_diag.so")
    L = _capi.load()
    _capi.set_kernel({"auto": _capi.KERNEL_AUTO, "general": _capi.KERNEL_GENERAL, "scan": _capi.KERNEL_SCAN, "inc": _capi.KERNEL_INC}[a.kernel])
    B, n, k = a.per_gpu, a.n, a.k
    m = int(round(a.alpha * n))
    icb, clb, lits, nv = cnf.uniform_ksat_device(B, n, m, k, seed=a.seed, device=dev)
    status = torch.zeros(B, dtype=torch.int32, device=dev)
    ctr = torch.zeros((B, 8), dtype=torch.int64, device=dev)
    sl = torch.zeros(B, dtype=torch.int32, device=dev)
    so = torch.zeros((B, max(n, 16)), dtype=torch.int32, device=dev)
    stride = max(n, 48)
    root_len = torch.zeros(B, dtype=torch.int32, device=dev)
    root = torch.zeros((B, stride), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    kern, lds, best = _capi.plan(n, m, m * k, k)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    resident = min(B, cus * best)
    for r in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        rc = L.satmi_dpll_batch_device(B, icb.data_ptr(), clb.data_ptr(), lits.data_ptr(), nv.data_ptr(), n, m,
                                       m * k, k, None, None, _capi.MODE_SOUND, 1, 0, 0.0, 1, stride, status.data_ptr(),
                                       ctr.data_ptr(), sl.data_ptr(), so.data_ptr(),
                                       root_len.data_ptr() if a.diag else None,
                                       root.data_ptr() if a.diag else None, st.cuda_stream)
        _capi.check(rc, "dpll")
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        c = ctr.cpu()
        ticks = c[:, 7].double()
        tick_s = 1e-8
        out = {"rep": r, "B": B, "n": n, "m": m, "lds_bytes": lds, "waves_per_cu": best, "resident_waves": resident,
               "kernel_ms": ms, "inst_per_s": B / ms * 1e3, "nodes": int(c[:, 0].sum()), "props": int(c[:, 2].sum()),
               "rounds": int(c[:, 6].sum()),
               "nodes_per_inst": float(c[:, 0].double().mean()), "max_nodes": int(c[:, 0].max()),
               "max_inst_ms": float(ticks.max()) * tick_s * 1e3, "mean_inst_ms": float(ticks.mean()) * tick_s * 1e3,
               "utilisation": float(ticks.sum()) * tick_s / (resident * ms * 1e-3),
               "wave_cycles_per_node_est": float(ticks.sum()) * tick_s * 2.1e9 / float(c[:, 0].sum()),
               "sat": int((c[:, 5] > 0).sum())}
        if a.diag:
            names = (("stage", "assign", "units", "conflict", "counts", "choose", "pure", "other")
                     if kern in (_capi.KERNEL_SCAN, _capi.KERNEL_INC) else
                     ("stage", "assign", "apply", "collect", "analyze", "pure", "backtrack", "other"))
            ph = root[:, :16].cpu().contiguous().view(torch.int64)[:, :8].double().sum(0)
            nodes = float(c[:, 0].sum())
            out["cycles_per_node"] = {nm: float(ph[i]) / nodes for i, nm in enumerate(names)}
            out["cycles_per_node"]["total"] = float(ph.sum()) / nodes
            out["rounds_per_node"] = float(c[:, 6].sum()) / nodes
            if kern in (_capi.KERNEL_SCAN, _capi.KERNEL_INC) and root.shape[1] >= 48:
                # path counts of the incremental unit scan (csrc/dpll_scan.hip inc_units, diag build)
                cn = root[:, :48].cpu().contiguous().view(torch.int64)[:, 8:24].double().sum(0)
                cnames = ("unit_scans", "fast_one_step", "fast_conflict", "fast_few_units", "units_found",
                          "general", "fast_bitmap", "batch_literals", "general_batch_gt16", "general_touched_gt64",
                          "fast_nun0", "fast_nun1", "fast_nun2", "fast_nun3_8", "propagate_calls", "assign_steps")
                out["per_node"] = {nm: float(cn[i]) / nodes for i, nm in enumerate(cnames)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
