"""Data-parallel gradient exchange (hvae/dist.py) over gloo, world_size 2, on CPU.

Checks the collective protocol the GPU path uses over RCCL: dense gradients are
averaged; row-sparse first-layer gradients of different lengths per rank are
gathered at the epoch's fixed size (max over ranks and batches, one host
all-reduce per epoch), weighted 1/world (0 past each rank's count) and merged
in (rank, slot) order, so every rank ends with the identical merged gradient =
mean of the ranks' dense grads.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N, H = 40, 8


class _Dense:
    def __init__(self, cap):
        self.cap = cap
        self.dense = torch.zeros(N, H, dtype=torch.float64)


def _cpu_merge(ex, items, grows, weights, out, rp):
    out.dense.zero_()
    for b in range(items.numel()):  # fixed (rank, slot) order, as the HIP merge
        out.dense[int(items[b])] += float(weights[b]) * grows[b].double()


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hvae.dist import DPExchange
    ex = DPExchange(dist.group.WORLD, torch.device("cpu"), N, H, merge_fn=_cpu_merge,
                    make_merged=lambda n, h, cap, dev: _Dense(cap))
    g = torch.Generator().manual_seed(100 + rank)
    small = torch.randn(1000, generator=g)
    mine = small.clone()
    ex.all_reduce_dense(small)
    # row-sparse: rank r touches 5 + 7 r sorted distinct items
    k = 5 + 7 * rank
    items = torch.sort(torch.randperm(N, generator=g)[:k]).values.int()
    cap = 32
    item_of = torch.zeros(cap, dtype=torch.int32)
    item_of[:k] = items
    rows = torch.zeros(cap, H)
    rows[:k] = torch.randn(k, H, generator=g)
    rows[k:] = 1e30  # stale slots beyond n_unique must never contribute
    ex.plan_epoch(np.array([3, k]))  # per-batch counts of this rank; the epoch size is the max over ranks
    assert ex.M == 5 + 7 * (world - 1)
    merged = ex.merged_rows(torch.tensor([k], dtype=torch.int32), item_of, rows)
    dense_mine = torch.zeros(N, H, dtype=torch.float64)
    dense_mine[items.long()] = rows[:k].double()
    q.put((rank, mine, small, dense_mine, merged.dense))
    dist.destroy_process_group()


def _worker_packed(rank, world, port, q):
    """The one-collective step: pack -> all_gather -> unpack_merge gives what all_reduce + exchange give."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hvae.dist import DPExchange
    ex = DPExchange(dist.group.WORLD, torch.device("cpu"), N, H, merge_fn=_cpu_merge,
                    make_merged=lambda n, h, cap, dev: _Dense(cap))
    g = torch.Generator().manual_seed(200 + rank)
    small = torch.randn(777, generator=g)
    mine = small.clone()
    k = 4 + 9 * rank
    items = torch.sort(torch.randperm(N, generator=g)[:k]).values.int()
    cap = 32
    item_of = torch.zeros(cap, dtype=torch.int32)
    item_of[:k] = items
    rows = torch.zeros(cap, H)
    rows[:k] = torch.randn(k, H, generator=g)
    rows[k:] = 1e30
    ex.plan_epoch(np.array([k, 2]))
    ex.pack(small, torch.tensor([k], dtype=torch.int32), item_of, rows)
    ex.communicate(small.numel())
    merged = ex.unpack_merge(small)
    dense_mine = torch.zeros(N, H, dtype=torch.float64)
    dense_mine[items.long()] = rows[:k].double()
    q.put((rank, mine, small, dense_mine, merged.dense.clone()))
    dist.destroy_process_group()


def test_dp_packed_exchange_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_packed, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mean_small = (res[0][1] + res[1][1]) / 2
    mean_dense = (res[0][3] + res[1][3]) / 2
    for _, _, small, _, merged in res:
        assert torch.allclose(small, mean_small, atol=1e-6)
        assert torch.allclose(merged, mean_dense, atol=1e-12)
    assert torch.equal(res[0][4], res[1][4]) and torch.equal(res[0][2], res[1][2])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_exchange_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mean_small = (res[0][1] + res[1][1]) / 2
    mean_dense = (res[0][3] + res[1][3]) / 2
    for _, _, small, _, merged in res:
        assert torch.allclose(small, mean_small, atol=1e-6)
        assert torch.allclose(merged, mean_dense, atol=1e-12)
    assert torch.equal(res[0][4], res[1][4]) and torch.equal(res[0][2], res[1][2])  # replicas identical
