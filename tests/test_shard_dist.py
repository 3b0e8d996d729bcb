"""Multi-rank path on CPU: instance sharding + verdict gather over `gloo`
(world_size 2 and 3), the same host logic bench.py / the GPU path use with RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from satmi import cnf
from satmi.shard import shard_range, solve_sharded, split_batch


def test_shard_range_partitions():
    for total in (0, 1, 7, 64, 262144, 262147):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
                assert e0 == b1
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_split_batch_roundtrip():
    batch = cnf.concat([cnf.uniform_ksat(5, 12, 30, 3, seed=1), cnf.pack([[[1, -2]], [], [[3]], [[1], [2, 3, -1]]])])
    got = []
    for r in range(3):
        part = split_batch(batch, 3, r)
        got += [part.instance(i) for i in range(part.num_instances)]
    assert got == [batch.instance(i) for i in range(batch.num_instances)]


def _oracle_solve(part):
    sat = np.zeros(part.num_instances, np.int8)
    ctr = np.zeros((part.num_instances, 8), np.int64)
    for i in range(part.num_instances):
        r = oracle.dpll(part.instance(i), "sound", max_solutions=1, sol_cap=1)
        sat[i] = 1 if r["counters"]["solutions"] else 0
        for j, k in enumerate(("nodes", "decisions", "unit_props", "pure_assigns", "conflicts", "solutions")):
            ctr[i, j] = r["counters"][k]
    return torch.from_numpy(sat), torch.from_numpy(ctr)


def _worker(rank, world, port, batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sat, tot = solve_sharded(batch, _oracle_solve)
        q.put((rank, sat.numpy().tolist(), tot.numpy().tolist()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_solve_sharded_gloo(world):
    batch = cnf.uniform_ksat(23, 20, 85, 3, seed=world)
    ref_sat, ref_ctr = _oracle_solve(batch)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, sat, tot in res:
        assert sat == ref_sat.numpy().tolist()
        assert tot == ref_ctr.sum(0).numpy().tolist()
