"""Instance sharding across ranks (one process per GPU) and the verdict gather.

The clause-set solving path partitions into independent formulas, so N GPUs
split a batch by instance index with no data-path collective; the only
exchange is the final gather of verdicts and counters (RCCL all-reduce /
all-gather over xGMI on MI355X, `gloo` in the CPU tests).

    shard_range(total, world, rank) -> (begin, end)     contiguous, sizes differ by <= 1
    gather_verdicts(local_sat, local_ctr, ...)          all-gather per-instance SAT flags,
                                                        all-reduce counter totals
"""
from typing import Optional, Tuple

import numpy as np


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Instances [begin, end) of `rank`: the first total % world ranks take one extra."""
    if world < 1 or not 0 <= rank < world or total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def gather_verdicts(local_sat, local_counters, total: int, group=None, device=None):
    """Collect every rank's per-instance verdicts (int8, 1 = SAT) into a [total]
    array on every rank and sum the [8] counter totals.

    `local_sat` / `local_counters` are torch tensors on this rank's device
    (int8 [shard], int64 [shard, 8]).  Ranks hold contiguous shards in rank
    order (shard_range), so the all-gather is a concatenation."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    dev = device if device is not None else local_sat.device
    tot = local_counters.sum(dim=0).to(torch.int64)
    if world == 1:
        return local_sat.clone(), tot
    # pad every shard to the largest size so the collective is rectangular
    sizes = [shard_range(total, world, r) for r in range(world)]
    cap = max(e - b for b, e in sizes)
    buf = torch.zeros(cap, dtype=torch.int8, device=dev)
    buf[:local_sat.numel()] = local_sat
    parts = [torch.zeros(cap, dtype=torch.int8, device=dev) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    dist.all_reduce(tot, group=group)
    out = torch.cat([parts[r][:e - b] for r, (b, e) in enumerate(sizes)])
    assert out.numel() == total and rank < world
    return out, tot


def split_batch(batch, world: int, rank: int):
    """This rank's CnfBatch slice of a host batch (contiguous instance range)."""
    from .cnf import CnfBatch

    b, e = shard_range(batch.num_instances, world, rank)
    icb = batch.inst_clause_begin.astype(np.int64)
    clb = batch.clause_lit_begin.astype(np.int64)
    c0, c1 = int(icb[b]), int(icb[e])
    l0, l1 = int(clb[c0]), int(clb[c1])
    lits = batch.lits[l0:l1] if l1 > l0 else np.zeros(1, np.int32)
    return CnfBatch((icb[b:e + 1] - c0).astype(np.int32), (clb[c0:c1 + 1] - l0).astype(np.int32),
                    np.ascontiguousarray(lits, dtype=np.int32), batch.inst_nvars[b:e].copy())


def solve_sharded(batch, solve_fn, group=None, device: Optional[object] = None):
    """Solve a host batch over all ranks: each rank runs `solve_fn(CnfBatch) ->
    (sat int8 [n], counters int64 [n, 8])` (torch tensors) on its shard, then the
    verdicts are gathered.  Returns (sat[total], counter_totals[8]) on every rank."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    part = split_batch(batch, world, rank)
    sat, ctr = solve_fn(part)
    return gather_verdicts(sat, ctr, batch.num_instances, group=group, device=device)
