"""Data-parallel sharding and exchange (hvae/dist.py) on CPU, the exchange over gloo with world size 2.

dp_shard: every step's union over the ranks is exactly one global batch of a permutation every rank draws
from the same seed (so a W-rank step is a single-GPU step over W B users), every user is visited once per
epoch, and every rank runs the same number of steps (no mismatched collectives, ADVICE r1: unequal shards).

The exchange (the same protocol the GPU path runs over RCCL, with CPU stand-ins for the two HIP kernels):
each rank packs [small dense gradients * w_r | its batch as compact CSR, values * w_r] and its first-layer
pre-activation gradient da; after the all-gathers every rank holds sum_r w_r g_r and the first-layer weight
gradient of the union batch, sum_r w_r sum_b x_bj da_b, identically. Checked for equal batches (w = 1 / W)
and for the uneven last batch (w_r = B_r / T, one rank possibly empty).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hvae.dist import dp_shard

N, H = 40, 8


@pytest.mark.parametrize("n,B,W", [(1000, 32, 2), (1000, 32, 3), (96, 32, 3), (10, 4, 4), (7, 64, 2), (4096, 64, 8)])
def test_dp_shard_union_is_global_batch(n, B, W):
    order = np.random.default_rng(n + B + W).permutation(n) + 1000
    parts = [dp_shard(order, B, W, r) for r in range(W)]
    n_full = parts[0][1]
    counts = parts[0][2]
    assert all(p[1] == n_full and p[2] == counts for p in parts)  # same steps, same collectives everywhere
    assert n_full == n // (W * B) and sum(counts) == n - n_full * W * B and max(counts) - min(counts) <= 1
    for g in range(n_full):  # step g: the ranks' batches, concatenated in rank order, = global batch g
        union = np.concatenate([p[0][g * B:(g + 1) * B] for p in parts])
        assert np.array_equal(union, order[g * W * B:(g + 1) * W * B])
    tail = np.concatenate([p[0][n_full * B:] for p in parts])
    assert np.array_equal(tail, order[n_full * W * B:])
    assert sorted(np.concatenate([p[0] for p in parts]).tolist()) == sorted(order.tolist())


def _cpu_pack(ex, x, weight, rp_out, col_out, val_out, cap):
    """hvae_csr_batch_pack on CPU: x = (indptr, indices, values, rows)."""
    indptr, indices, values, rows = x
    e = 0
    rp_out[0] = 0
    for j, r in enumerate(rows):
        for k in range(indptr[r], indptr[r + 1]):
            col_out[e] = int(indices[k])
            val_out[e] = float(weight) * float(values[k])
            e += 1
        rp_out[j + 1] = e


class _Dense:
    def __init__(self):
        self.dense = torch.zeros(N, H, dtype=torch.float64)


def _cpu_merge(ex, row_ptr, col_idx, vals, rows, nb, da, out):
    """hvae_w1_rowgrad on CPU: sum over the union batch's rows, in batch order."""
    out.dense.zero_()
    for i in range(nb):
        r = int(rows[i])
        for e in range(int(row_ptr[r]), int(row_ptr[r + 1])):
            out.dense[int(col_idx[e])] += float(vals[e]) * da[i].double()


def _batch(rng, nb):
    lens = rng.integers(1, 6, size=nb)
    indptr = np.concatenate([[0], np.cumsum(lens)])
    indices = np.concatenate([np.sort(rng.choice(N, size=l, replace=False)) for l in lens])
    values = rng.integers(1, 3, size=int(indptr[-1])).astype(np.float32)
    return indptr, indices, values


def _worker(rank, world, port, q, B, sizes):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hvae.dist import DPExchange
    ns = 777
    ex = DPExchange(dist.group.WORLD, torch.device("cpu"), N, H, ns, pack_fn=_cpu_pack, merge_fn=_cpu_merge,
                    make_merged=lambda n, h, cap, dev: _Dense())
    rng = np.random.default_rng(300 + rank)
    nb = sizes[rank]
    T = sum(sizes)
    indptr, indices, values = _batch(rng, max(nb, 1))
    g_small = torch.as_tensor(rng.standard_normal(ns).astype(np.float32))
    da = torch.as_tensor(rng.standard_normal((max(nb, 1), H)).astype(np.float32))
    mine = (g_small.clone(), indptr, indices, values, da.clone())
    ex.plan(B, 5 * B)
    w = nb / T
    if nb:
        ex.pack(g_small, (indptr, indices, values, list(range(nb))), nb, da, w)
    else:
        ex.pack(g_small, None, 0, None, 0.0)
    ex.communicate()
    merged = ex.unpack_merge(g_small)
    # numpy, not tensors: a tensor crosses the queue as a file descriptor the exiting worker may close before the
    # parent receives it (ConnectionResetError in the parent's rebuild)
    q.put((rank, tuple(x.numpy().copy() if torch.is_tensor(x) else x for x in mine), g_small.numpy().copy(),
           merged.dense.numpy().copy()))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("B,sizes", [(6, [6, 6]), (6, [5, 4]), (3, [1, 0])])
def test_dp_exchange_gloo_world2(B, sizes):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, B, sizes)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    res = [(r, tuple(torch.as_tensor(x) if i in (0, 4) else x for i, x in enumerate(m)), torch.as_tensor(sm), torch.as_tensor(w)) for r, m, sm, w in res]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T = sum(sizes)
    want_small = sum((sizes[r] / T) * res[r][1][0].double() for r in range(world))
    want_w1 = torch.zeros(N, H, dtype=torch.float64)
    for r in range(world):  # the union batch, rank-major: sum_b w_r x_bj da_b
        _, (g, indptr, indices, values, da), _, _ = res[r]
        for b in range(sizes[r]):
            for k in range(indptr[b], indptr[b + 1]):
                want_w1[indices[k]] += (sizes[r] / T) * float(values[k]) * da[b].double()
    for _, _, small, w1 in res:
        assert torch.allclose(small.double(), want_small, atol=1e-6)
        assert torch.allclose(w1, want_w1, atol=1e-6)
    assert torch.equal(res[0][2], res[1][2]) and torch.equal(res[0][3], res[1][3])  # replicas identical
