"""bench.py's multi-rank workload on CPU: a rank's shard of the chunked bench
batch is exactly the same slice of the world-1 batch for every rank count (so
an N-GPU run solves the instances the 1-GPU run solves), and the verdict
gather + hash agrees across world sizes over `gloo` (RCCL on the GPU box)."""
import hashlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from satmi.shard import gather_verdicts, shard_range

N, M, K = 20, 85, 3


def _whole(total, seed):
    return bench.chunked_batch(0, total, N, M, K, seed, torch.device("cpu"))


@pytest.mark.parametrize("total", [bench.CHUNK * 2 + 37, 3 * bench.CHUNK])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_rank_shards_are_slices_of_the_world1_batch(total, world):
    icb, clb, lits, nv = _whole(total, seed=11)
    assert icb.numel() == total + 1 and lits.numel() == total * M * K and nv.numel() == total
    for r in range(world):
        b0, b1 = shard_range(total, world, r)
        s_icb, s_clb, s_lits, s_nv = bench.chunked_batch(b0, b1, N, M, K, 11, torch.device("cpu"))
        assert torch.equal(s_lits, lits[b0 * M * K:b1 * M * K])
        assert torch.equal(s_icb, icb[:b1 - b0 + 1]) and torch.equal(s_clb, clb[:(b1 - b0) * M + 1])
        assert torch.equal(s_nv, nv[b0:b1])


def test_batches_differ_per_stream_and_chunk():
    a = _whole(bench.CHUNK * 2, seed=bench.batch_seed(5, 0))[2].view(2, -1)
    b = _whole(bench.CHUNK * 2, seed=bench.batch_seed(5, 1))[2].view(2, -1)
    assert not torch.equal(a[0], a[1]) and not torch.equal(a[0], b[0])


def test_span_union():
    hz = 1000.0   # ticks of 1 ms
    assert bench.span_union_ms([(0, 10), (5, 12), (20, 25)], hz) == pytest.approx(17.0)
    assert bench.span_union_ms([(0, 10)], hz) == pytest.approx(10.0)


def _verdicts(total):
    # a deterministic stand-in verdict per instance of the virtual batch
    return (torch.arange(total) * 2654435761 % 7 < 3).to(torch.int8)


def _worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b0, b1 = shard_range(total, world, rank)
        local = _verdicts(total)[b0:b1].clone()
        ctr = torch.ones((b1 - b0, 8), dtype=torch.int64)
        out, tot = gather_verdicts(local, ctr, total)
        q.put((rank, hashlib.sha256(out.numpy().tobytes()).hexdigest()[:16], tot.tolist()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_verdict_hash_same_for_every_world(world):
    total = 1001
    want = hashlib.sha256(_verdicts(total).numpy().tobytes()).hexdigest()[:16]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, sha, tot in res:
        assert sha == want
        assert tot == [total] * 8
