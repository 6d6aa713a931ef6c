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
So a step has no host synchronisation: two captured graphs (forward/backward;
merge/clip/Adam) with the three collectives launched between them. Entries
past a rank's own count carry weight 0.

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
