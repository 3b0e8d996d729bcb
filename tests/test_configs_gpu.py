"""BASELINE configs[2] at its full size on the GPU: 262,144 uniform random 3-SAT
instances of n=100, alpha=4.26, generated in HBM by the bench's own generator
and solved through the device-pointer C ABI (satmi_dpll_batch_device) exactly as
bench.py does.  Checks: every status is a finished search, every model satisfies
every clause of its formula (on the device, all instances), and a sample of SAT
and UNSAT instances equals the CPU oracle bit for bit (every counter, the model)."""
import numpy as np
import pytest

import oracle
from satmi import _capi, cnf

pytestmark = pytest.mark.gpu
CTR = ("nodes", "decisions", "unit_props", "pure_assigns", "conflicts", "solutions")


def test_configs2_full_batch_device():
    import torch
    dev = torch.device("cuda", 0)
    L = _capi.load()
    B, n, k = 262144, 100, 3
    m = int(round(4.26 * n))
    icb, clb, lits, nv = cnf.uniform_ksat_device(B, n, m, k, seed=20261016, device=dev)
    status = torch.zeros(B, dtype=torch.int32, device=dev)
    counters = torch.zeros((B, _capi.NCOUNTERS), dtype=torch.int64, device=dev)
    sol_len = torch.zeros(B, dtype=torch.int32, device=dev)
    sol_lits = torch.zeros((B, n), dtype=torch.int32, device=dev)
    rc = L.satmi_dpll_batch_device(B, icb.data_ptr(), clb.data_ptr(), lits.data_ptr(), nv.data_ptr(), n, m, m * k, k,
                                   None, None, _capi.MODE_SOUND, 1, 0, 0.0, 1, n, status.data_ptr(),
                                   counters.data_ptr(), sol_len.data_ptr(), sol_lits.data_ptr(), None, None, None)
    _capi.check(rc, "satmi_dpll_batch_device")
    torch.cuda.synchronize()
    ok = (status == _capi.DPLL_STOPPED) | (status == _capi.DPLL_EXHAUSTED)
    assert bool(ok.all())
    sat = counters[:, 5] > 0
    assert bool(((status == _capi.DPLL_STOPPED) == sat).all())
    # every model satisfies every clause (all 262,144 instances, on the device)
    val = torch.zeros((B, n + 1), dtype=torch.int8, device=dev)
    live = torch.arange(n, device=dev)[None, :] < sol_len[:, None]
    idx = torch.where(live, sol_lits.abs(), 0).to(torch.int64)
    val.scatter_(1, idx, torch.where(sol_lits > 0, 1, -1).to(torch.int8))
    val[:, 0] = 0
    lv = lits.view(B, m, k).to(torch.int64)
    litval = torch.gather(val, 1, lv.abs().view(B, -1)).view(B, m, k) * torch.sign(lv).to(torch.int8)
    clause_ok = (litval > 0).any(dim=2).all(dim=1)
    assert bool(((~sat) | clause_ok).all())
    frac = float(sat.float().mean())
    assert 0.4 < frac < 0.7, frac   # near the threshold about half the instances are SAT
    # bit-exact against the oracle on 12 SAT + 12 UNSAT instances spread over the batch
    sat_h, st_h = sat.cpu().numpy(), status.cpu().numpy()
    ctr_h, sl_h, so_h = counters.cpu().numpy(), sol_len.cpu().numpy(), sol_lits.cpu().numpy()
    host = cnf.CnfBatch(icb.cpu().numpy(), clb.cpu().numpy(), lits.cpu().numpy(), nv.cpu().numpy())
    rng = np.random.default_rng(7)
    pick = list(rng.choice(np.flatnonzero(sat_h), 12, replace=False)) + \
        list(rng.choice(np.flatnonzero(~sat_h), 12, replace=False))
    for b in pick:
        o = oracle.dpll(host.instance(int(b)), "sound", max_solutions=1, sol_cap=1)
        for j, key in enumerate(CTR):
            assert int(ctr_h[b, j]) == o["counters"][key], (int(b), key)
        assert int(st_h[b]) == (_capi.DPLL_STOPPED if o["status"] == 1 else _capi.DPLL_EXHAUSTED)
        if sat_h[b]:
            assert so_h[b, :sl_h[b]].tolist() == o["solutions"][0]
