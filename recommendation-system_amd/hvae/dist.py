"""User-batch data parallelism for the fused trainer (one process per GPU, RCCL over xGMI).

The reference is single-device (no collectives anywhere). The
MI355X build shards users across ranks; parameters, Adam state and the frozen
embeddings are replicated (E is never communicated). After each rank's
forward/backward:

  * the small dense gradients (every parameter except the first-layer
    weight, ~0.3-0.8 M floats) are all-reduced with ReduceOp.AVG;
  * the first-layer weight gradient is row-sparse (only the items of each
    rank's batch): every rank all-gathers the (item id, gradient row) lists
    of all ranks and merges them with the same deterministic counting-sort
    kernel that builds the local rows (hvae_w1_rowgrad), weighting each rank
    by 1/world. A dense all-reduce of the [N, H] gradient would move N*H*4
    bytes per step instead.

The row lists are exchanged at a fixed size M per epoch: every rank counts the
unique items of each of its batches on the host when the epoch order is drawn,
and one all-reduce(MAX) per epoch gives the largest list of any rank and batch.
Entries past a rank's own count carry weight 0.

A step then makes ONE collective: each rank packs [dense gradients | row count |
item ids | gradient rows] into one fp32 buffer at the end of its forward/backward
graph, a single all_gather_into_tensor moves it (per-collective latency, not
bytes, dominates at these sizes on xGMI), and the update graph averages the
dense parts in rank order and merges the row lists. So a step has no host
synchronisation: two captured graphs with one collective between them.

Then every rank clips and steps Adam on identical gradients, so the replicas
stay bit-identical. The merge function is injectable so that the collective
protocol can be tested with gloo on CPU (tests/test_dist_gloo.py); with the
gloo backend, device tensors are staged through host memory.
"""
from __future__ import annotations

from typing import Callable

import numpy as np
import torch
import torch.distributed as dist


def batch_unique_counts(indptr: np.ndarray, indices: np.ndarray, order: np.ndarray, B: int,
                        drop_last: bool = False) -> np.ndarray:
    """Unique items of each batch of `order` (users, batch size B): the host twin of the plan kernels."""
    n = len(order)
    nb = n // B if drop_last else -(-n // B)
    out = np.zeros(nb, dtype=np.int64)
    for b in range(nb):
        us = order[b * B:(b + 1) * B]
        parts = [indices[indptr[u]:indptr[u + 1]] for u in us]
        out[b] = len(np.unique(np.concatenate(parts))) if parts else 0
    return out


class DPExchange:
    def __init__(self, group, device: torch.device, n_items: int, H: int,
                 merge_fn: Callable | None = None, make_merged: Callable | None = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        self.backend = dist.get_backend(group)
        self.n_items, self.H = n_items, H
        self.merge_fn = merge_fn or _hip_merge
        self.make_merged = make_merged or _hip_make_merged
        self.M = 0
        self._merged = None
        self._buf = None
        self._pk = None

    # -- collectives (gloo cannot take device tensors for every op: stage through host) --
    def _stage(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu() if (self.backend == "gloo" and t.device.type != "cpu") else t

    def all_reduce_dense(self, g: torch.Tensor) -> None:
        if self.world == 1:
            return
        x = self._stage(g)
        op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
        dist.all_reduce(x, op=op, group=self.group)
        if op != dist.ReduceOp.AVG:
            x.div_(self.world)
        if x is not g:
            g.copy_(x)

    def _all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        o, i = self._stage(out), self._stage(inp)
        dist.all_gather_into_tensor(o, i, group=self.group)
        if o is not out:
            out.copy_(o)

    # -- one-collective step: pack (graph 1) -> all-gather (eager) -> unpack + merge (graph 2) --
    def _packed(self, n_small: int):
        """(send [L], recv [W, L]) for the epoch's M; L = n_small + 1 + M + M * H (fp32 words)."""
        M, W, H = self.M, self.world, self.H
        L = n_small + 1 + M + M * H
        if self._pk is None or self._pk[0].numel() != L:
            self._pk = (torch.zeros(L, dtype=torch.float32, device=self.device),
                        torch.zeros(W, L, dtype=torch.float32, device=self.device))
        return self._pk

    def pack(self, g_small: torch.Tensor, n_unique: torch.Tensor, item_of: torch.Tensor, rows: torch.Tensor) -> None:
        """Device copies of this rank's step gradients into the send buffer (capturable)."""
        M, ns = self.M, g_small.numel()
        assert M > 0, "plan_epoch() first"
        assert item_of.numel() >= M and rows.shape[0] >= M, "row-gradient buffers shorter than the exchange size"
        send, _ = self._packed(ns)
        send[:ns].copy_(g_small.reshape(-1))
        send[ns:ns + 1].view(torch.int32).copy_(n_unique.reshape(1).to(torch.int32))
        send[ns + 1:ns + 1 + M].view(torch.int32).copy_(item_of[:M])
        send[ns + 1 + M:].view(M, self.H).copy_(rows[:M])

    def communicate(self, n_small: int) -> None:
        """The step's one collective (eager, between the two graphs)."""
        send, recv = self._packed(n_small)
        if self.world == 1:
            recv[0].copy_(send)
            return
        self._all_gather(recv.reshape(-1), send)

    def unpack_merge(self, g_small: torch.Tensor):
        """Dense gradients <- mean over ranks (summed in rank order); row lists -> merged row gradient."""
        M, W, H, ns = self.M, self.world, self.H, g_small.numel()
        _, recv = self._packed(ns)
        torch.sum(recv[:, :ns], dim=0, out=g_small.reshape(-1))
        g_small.div_(W)
        b = self._buf
        b["n"].copy_(recv[:, ns].contiguous().view(torch.int32))
        b["items"].view(W, M).copy_(recv[:, ns + 1:ns + 1 + M].contiguous().view(torch.int32))
        b["rows"].view(W, M, H).copy_(recv[:, ns + 1 + M:].reshape(W, M, H))
        return self.merge()

    def plan_epoch(self, counts_per_batch: np.ndarray) -> int:
        """One host collective per epoch: the largest row list of any rank and batch. (Re)allocates the
        exchange and merge buffers when it grows, so that nothing is allocated inside a captured step."""
        m = torch.tensor([int(counts_per_batch.max()) if len(counts_per_batch) else 1], dtype=torch.int64,
                         device=self.device if self.backend == "nccl" else "cpu")  # RCCL takes device tensors only
        if self.world > 1:
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        M = max(int(m.item()), 1)
        if M > self.M:
            self.M = M
            W, H, dev = self.world, self.H, self.device
            self._buf = {
                "n": torch.zeros(W, dtype=torch.int32, device=dev),
                "items": torch.zeros(W * M, dtype=torch.int32, device=dev),
                "rows": torch.zeros(W * M, H, dtype=torch.float32, device=dev),
                "w": torch.zeros(W * M, dtype=torch.float32, device=dev),
                "rp": torch.arange(W * M + 1, dtype=torch.int64, device=dev),
                "j": torch.arange(M, dtype=torch.int32, device=dev),
            }
            self._merged = self.make_merged(self.n_items, H, W * M, dev)
            self._pk = None
        return self.M

    def exchange(self, n_unique: torch.Tensor, item_of: torch.Tensor, rows: torch.Tensor) -> None:
        """The collectives of a step: all-gather every rank's row list at the epoch's fixed size M."""
        M = self.M
        assert M > 0, "plan_epoch() first"
        assert item_of.numel() >= M and rows.shape[0] >= M, "row-gradient buffers shorter than the exchange size"
        b = self._buf
        self._all_gather(b["n"], n_unique.reshape(1).to(torch.int32))
        self._all_gather(b["items"], item_of[:M].contiguous())
        self._all_gather(b["rows"], rows[:M].contiguous())

    def merge(self):
        """Device-only (graph-capturable) half: weights 1/W for each rank's own entries, 0 past its count
        (those point at item 0), then the deterministic merge into the merged row gradient."""
        W = self.world
        b = self._buf
        valid = (b["j"][None, :] < b["n"][:, None]).reshape(-1)  # rank-major [W*M]
        torch.div(valid.to(torch.float32), W, out=b["w"])
        b["items"].masked_fill_(~valid, 0)
        self.merge_fn(self, b["items"], b["rows"], b["w"], self._merged, b["rp"])
        return self._merged

    def merged_rows(self, n_unique, item_of, rows):
        self.exchange(n_unique, item_of, rows)
        return self.merge()


def _hip_make_merged(n_items, H, cap, device):
    from . import ops
    return ops.RowGradBuffers(n_items, H, cap, device)


def _hip_merge(ex: DPExchange, items, grows, weights, out, rp):
    """Sum the gathered rows per item in (rank, slot) order with hvae_w1_rowgrad."""
    from . import ops
    csr = ops.Csr(rp, items.to(torch.int32), weights, ex.n_items)
    ops.w1_rowgrad(csr, grows, out)
