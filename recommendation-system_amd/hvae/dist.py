"""User-batch data parallelism for the fused trainer (one process per GPU, RCCL over xGMI).

The reference is single-device (no collectives anywhere). The
MI355X build shards users across ranks; parameters, Adam state and the frozen
embeddings are replicated (E is never communicated). After each rank's
forward/backward:

  * the small dense gradients (every parameter except the first-layer
    weight, ~0.3-0.8 M floats) are all-reduced with ReduceOp.AVG;
  * the first-layer weight gradient is row-sparse (only the items of each
    rank's batch): every rank all-gathers the (item id, gradient row) lists
    of all ranks -- padded to the largest count -- and merges them with the
    same deterministic counting-sort kernel that builds the local rows
    (hvae_w1_rowgrad), weighting each rank by 1/world. A dense all-reduce of
    the [N, H] gradient would move N*H*4 bytes per step instead.

Then every rank clips and steps Adam on identical gradients, so the replicas
stay bit-identical. The merge function is injectable so that the collective
protocol can be tested with gloo on CPU (tests/test_dist_gloo.py).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


class DPExchange:
    def __init__(self, group, device: torch.device, n_items: int, H: int,
                 merge_fn: Callable | None = None, make_merged: Callable | None = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        self.n_items, self.H = n_items, H
        self.merge_fn = merge_fn or _hip_merge
        self.make_merged = make_merged or _hip_make_merged
        self._merged = None
        self._rowptr: dict[int, torch.Tensor] = {}

    def all_reduce_dense(self, g: torch.Tensor) -> None:
        if self.world > 1:
            op = dist.ReduceOp.AVG if dist.get_backend(self.group) == "nccl" else dist.ReduceOp.SUM
            dist.all_reduce(g, op=op, group=self.group)
            if op != dist.ReduceOp.AVG:
                g.div_(self.world)

    def gather_rows(self, n_unique: torch.Tensor, item_of: torch.Tensor, rows: torch.Tensor):
        """All-gather the row-sparse lists. Returns (items [W*M], rows [W*M, H], weights [W*M])."""
        W = self.world
        counts = [torch.zeros_like(n_unique) for _ in range(W)]
        dist.all_gather(counts, n_unique, group=self.group)
        cnt = [int(c.item()) for c in counts]  # host sync: sizes of the variable-length exchange
        M = max(max(cnt), 1)
        items = torch.empty(W * M, dtype=item_of.dtype, device=item_of.device)
        grows = torch.empty(W * M, self.H, dtype=rows.dtype, device=rows.device)
        dist.all_gather_into_tensor(items, item_of[:M].contiguous(), group=self.group)
        dist.all_gather_into_tensor(grows, rows[:M].contiguous(), group=self.group)
        w = torch.zeros(W, M, dtype=torch.float32)
        for r, c in enumerate(cnt):
            w[r, :c] = 1.0 / W
        items_v = items.view(W, M).clone()
        for r, c in enumerate(cnt):  # padding entries point at item 0 with weight 0 (no contribution)
            items_v[r, c:] = 0
        return items_v.reshape(-1), grows, w.reshape(-1).to(rows.device), M

    def merged_rows(self, n_unique, item_of, rows):
        items, grows, weights, M = self.gather_rows(n_unique, item_of, rows)
        cap = self.world * M
        if self._merged is None or self._merged.cap < cap:
            self._merged = self.make_merged(self.n_items, self.H, max(cap, 1), self.device)
        self.merge_fn(self, items, grows, weights, self._merged)
        return self._merged


def _hip_make_merged(n_items, H, cap, device):
    from . import ops
    return ops.RowGradBuffers(n_items, H, cap, device)


def _hip_merge(ex: DPExchange, items, grows, weights, out):
    """Sum the gathered rows per item in (rank, slot) order with hvae_w1_rowgrad."""
    from . import ops
    n = items.numel()
    rp = ex._rowptr.get(n)
    if rp is None:
        rp = torch.arange(n + 1, dtype=torch.int64, device=items.device)
        ex._rowptr[n] = rp
    csr = ops.Csr(rp, items.to(torch.int32), weights, ex.n_items)
    ops.w1_rowgrad(csr, grows, out)
