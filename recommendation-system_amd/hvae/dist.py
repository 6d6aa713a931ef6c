"""User-batch data parallelism for the fused trainer (one process per GPU, RCCL over xGMI).

The reference is single-device (no collectives anywhere). The MI355X build shards users across
ranks; parameters, Adam state and the frozen embeddings are replicated (E is never communicated), and one
data-parallel step is one step of the single-GPU trainer over the UNION of the ranks' batches:

  * sharding (dp_shard): every rank draws the same seeded permutation of all users; global batch g is users
    [g W B, (g + 1) W B) of it and rank r takes the r-th B of them, so the union of a step is exactly the
    global batch one GPU would take at batch size W B. The last, partial global batch is split over the ranks
    as evenly as possible (a rank may get none). Every rank therefore runs the same number of steps, with
    the same collectives (pre-sharded data, as bench.py's per-rank shards, must have equal sizes).
  * exchange (one step, two all-gathers): rank r's packet is [its dense small-parameter gradient * w_r | its
    batch compacted as CSR (row offsets, item ids, values * w_r)] plus its da [B, H], the gradient of the
    first hidden layer's pre-activation, with w_r = B_r / (sum of the ranks' B_r) (1 / W for full batches).
    The first-layer weight gradient is linear in (x, da): every rank rebuilds it for the union batch from the
    gathered packets with the same deterministic row-gradient kernels, in rank-major batch order -- the order
    one GPU would use for the union batch. Per rank B H + 2 nnz + B words move instead of (distinct items)
    x H (Syn-10M: ~9 MB instead of ~160 MB), and nothing is padded to an epoch maximum.
  * the dense small gradients are summed in rank order; every rank then clips and steps Adam on identical
    gradients, so the replicas stay bit-identical.

In the fused trainer a step is two captured graphs (forward/backward + pack; unpack + union row gradient +
clip + Adam) with the two collectives launched eagerly between them. pack_fn / merge_fn are injectable so
that the protocol runs with gloo on CPU (tests/test_dist_gloo.py); with the gloo backend device tensors are
staged through host memory.
"""
from __future__ import annotations

import os
from typing import Callable

import numpy as np
import torch
import torch.distributed as dist


def init_from_env(backend: str | None = None):
    """torchrun's environment (WORLD_SIZE, RANK, LOCAL_RANK, MASTER_*) -> one process per GPU: select GPU
    LOCAL_RANK and join the process group (RCCL -- backend "nccl" on ROCm -- unless HVAE_DIST_BACKEND names
    another) before any other GPU work. Returns the group, or None for a single process."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(torch.cuda.device_count(), 1)
    dev = torch.device("cuda", local % ndev)  # more ranks than GPUs: a one-GPU rehearsal (gloo)
    torch.cuda.set_device(dev)
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        be = backend or os.environ.get("HVAE_DIST_BACKEND", "nccl")
        if be == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(be)
    return dist.group.WORLD


def is_main(group) -> bool:
    return group is None or dist.get_rank(group) == 0


def all_reduce_host(values, group, device, op=dist.ReduceOp.SUM) -> np.ndarray:
    """Host numbers reduced over the ranks (a device tensor for RCCL, a CPU one for gloo)."""
    t = torch.as_tensor(np.asarray(values, dtype=np.float64),
                        device=device if dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(t, op=op, group=group)
    return t.cpu().numpy()


def broadcast_seed(group, device) -> int:
    """A seed drawn from rank 0's numpy global RNG, the same on every rank."""
    s = np.array([np.random.randint(0, 2 ** 31 - 1) if dist.get_rank(group) == 0 else 0], dtype=np.float64)
    t = torch.as_tensor(s, device=device if dist.get_backend(group) == "nccl" else "cpu")
    dist.broadcast(t, 0, group=group)
    return int(t.cpu().item())


def dp_shard(order: np.ndarray, B: int, world: int, rank: int):
    """This rank's users for one epoch of `order` (a permutation of all users, identical on every rank).

    Returns (users, n_full, tail_counts): the rank's users in step order (n_full full batches of B, then its
    tail), the number of full global batches, and every rank's share of the last partial global batch.
    """
    order = np.asarray(order)
    WB = world * B
    n = len(order)
    n_full = n // WB
    T = n - n_full * WB
    counts = [T // world + (1 if r < T % world else 0) for r in range(world)]
    full = order[: n_full * WB].reshape(n_full, world, B)[:, rank, :].reshape(-1)
    start = n_full * WB + sum(counts[:rank])
    return np.concatenate([full, order[start:start + counts[rank]]]), n_full, counts


class DPExchange:
    def __init__(self, group, device: torch.device, n_items: int, H: int, n_small: int,
                 pack_fn: Callable | None = None, merge_fn: Callable | None = None,
                 make_merged: Callable | None = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        self.backend = dist.get_backend(group)
        self.n_items, self.H, self.ns = n_items, H, n_small
        self.pack_fn = pack_fn or _hip_pack
        self.merge_fn = merge_fn or _hip_merge
        self.make_merged = make_merged or _hip_make_merged
        self.B = self.cap = 0
        # set by hvae_csr_batch_pack when a batch held more entries than its packet's cap (checked by check())
        self.overflow = torch.zeros(1, dtype=torch.int32, device=device)
        self._plans: dict = {}
        self._merged: dict = {}

    def check(self) -> None:
        """Raise if any packet since the last check dropped entries (its cap, sized from the host CSR, was
        exceeded): the union row gradient of that step would be wrong. One host read, at epoch end."""
        if int(self.overflow.item()):
            self.overflow.zero_()
            raise RuntimeError("data-parallel packet overflow: a batch held more CSR entries than its cap")

    # ----------------------------------------------------------- collectives ---
    def _stage(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu() if (self.backend == "gloo" and t.device.type != "cpu") else t

    def _all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        o, i = self._stage(out), self._stage(inp)
        dist.all_gather_into_tensor(o, i, group=self.group)
        if o is not out:
            out.copy_(o)

    def all_reduce(self, values, op=dist.ReduceOp.SUM) -> np.ndarray:
        """Host values reduced over the ranks (epoch bookkeeping, not per step)."""
        t = torch.as_tensor(np.asarray(values, dtype=np.float64),
                            device=self.device if self.backend == "nccl" else "cpu")  # RCCL takes device tensors
        if self.world > 1:
            dist.all_reduce(t, op=op, group=self.group)
        return t.cpu().numpy()

    # ------------------------------------------------------------- buffers ---
    def plan(self, B: int, cap: int) -> None:
        """Select the buffers of a step of B users per rank whose packed batch holds at most cap entries (the
        same B and cap on every rank). Each (B, cap) keeps its own buffers for the life of the exchange, so a
        graph captured against them stays valid when the epoch's short last step switches B and back."""
        key = (B, cap)
        if key not in self._plans:
            W, H, ns, dev = self.world, self.H, self.ns, self.device
            L = ns + (B + 1) + 2 * cap  # fp32 words: [g_small | row offsets | items | values]
            j = torch.arange(B, dtype=torch.int32, device=dev)
            if W * cap not in self._merged:  # the union batch's row gradient, per packet cap
                self._merged[W * cap] = self.make_merged(self.n_items, H, W * cap, dev)
            self._plans[key] = dict(
                L=L, off_rp=ns, off_col=ns + B + 1,
                send=torch.zeros(L, dtype=torch.float32, device=dev),
                recv=torch.zeros(W, L, dtype=torch.float32, device=dev),
                send_da=torch.zeros(B, H, dtype=torch.float32, device=dev),
                send_g=torch.zeros(ns, dtype=torch.float32, device=dev),
                recv_g=torch.zeros(W, ns, dtype=torch.float32, device=dev),
                recv_da=torch.zeros(W * B, H, dtype=torch.float32, device=dev),
                # the two-exchange step gathers the CSR part of the packet only (the small gradients travel in
                # their own exchange after the backward): [W][row offsets | items | values]
                recv_csr=torch.zeros(W, L - ns, dtype=torch.float32, device=dev),
                rp_u=torch.zeros(W * (B + 1), dtype=torch.int64, device=dev),
                base=(torch.arange(W, dtype=torch.int64, device=dev) * L + ns + B + 1)[:, None],
                base_csr=(torch.arange(W, dtype=torch.int64, device=dev) * (L - ns) + B + 1)[:, None],
                rows_u=(torch.arange(W, dtype=torch.int32, device=dev)[:, None] * (B + 1) + j[None, :]).reshape(-1),
                merged=self._merged[W * cap])
        for k, v in self._plans[key].items():
            setattr(self, k, v)
        self.B, self.cap = B, cap

    # ---------------------------------------------------------------- step ---
    def pack(self, g_small: torch.Tensor, x, nb: int, da: torch.Tensor | None, weight: float) -> None:
        """Device-only (graph-capturable): this rank's packet. x: its batch (CsrBatch of nb rows, or None
        when the rank has no users in this step); da: its [nb, H] pre-activation gradient."""
        ns = self.ns
        torch.mul(g_small.reshape(-1), weight, out=self.send[:ns])
        if x is None or nb == 0:
            self.send[ns:].zero_()
            self.send_da.zero_()
            return
        flat = self.send
        self.pack_fn(self, x, weight, flat[self.off_rp:self.off_rp + nb + 1].view(torch.int32),
                     flat[self.off_col:self.off_col + self.cap].view(torch.int32),
                     flat[self.off_col + self.cap:], self.cap)
        if nb < self.B:  # a short tail: rows past nb are empty
            flat[self.off_rp + nb + 1:self.off_rp + self.B + 1].view(torch.int32).copy_(
                flat[self.off_rp + nb:self.off_rp + nb + 1].view(torch.int32).expand(self.B - nb))
            self.send_da[nb:].zero_()
        if da is not None and da.data_ptr() != self.send_da.data_ptr():
            self.send_da[:nb].copy_(da[:nb])

    def communicate(self) -> None:
        """The step's collectives (eager, between the two graphs)."""
        if self.world == 1:
            self.recv[0].copy_(self.send)
            self.recv_da.copy_(self.send_da)
            return
        self._all_gather(self.recv.reshape(-1), self.send)
        self._all_gather(self.recv_da, self.send_da)

    # ------------------------------------------- the step in two exchanges ---
    # The trainer sends the batch CSR before the forward, so that the union batch's row-gradient plan (which
    # needs the batches only) runs on a side stream beside the forward / decoder, and the small gradients
    # and da after the backward; only the apply of the union row gradient is left between the second
    # exchange and Adam. The packets and the results are those of pack / communicate / unpack_merge.
    def pack_csr(self, x, nb: int, weight: float) -> None:
        """Device-only: this rank's batch as compact CSR (values * weight), before its forward."""
        flat = self.send
        if x is None or nb == 0:
            flat[self.ns:].zero_()
            return
        self.pack_fn(self, x, weight, flat[self.off_rp:self.off_rp + nb + 1].view(torch.int32),
                     flat[self.off_col:self.off_col + self.cap].view(torch.int32),
                     flat[self.off_col + self.cap:], self.cap)
        if nb < self.B:  # a short tail: rows past nb are empty
            flat[self.off_rp + nb + 1:self.off_rp + self.B + 1].view(torch.int32).copy_(
                flat[self.off_rp + nb:self.off_rp + nb + 1].view(torch.int32).expand(self.B - nb))

    def pack_grads(self, g_small: torch.Tensor, nb: int, da: torch.Tensor | None, weight: float) -> None:
        """Device-only: the weighted small gradients and da, after the backward."""
        torch.mul(g_small.reshape(-1), weight, out=self.send_g)
        if da is None or nb == 0:
            self.send_da.zero_()
            return
        if nb < self.B:
            self.send_da[nb:].zero_()
        if da.data_ptr() != self.send_da.data_ptr():
            self.send_da[:nb].copy_(da[:nb])

    def communicate_csr(self) -> None:
        csr = self.send[self.ns:]  # the packet past the small-gradient words (unused in this exchange)
        if self.world == 1:
            self.recv_csr[0].copy_(csr)
            return
        self._all_gather(self.recv_csr.reshape(-1), csr)

    def communicate_grads(self) -> None:
        if self.world == 1:
            self.recv_g[0].copy_(self.send_g)
            self.recv_da.copy_(self.send_da)
            return
        self._all_gather(self.recv_g.reshape(-1), self.send_g)
        self._all_gather(self.recv_da, self.send_da)

    def merge_plan(self) -> None:
        """Device-only, on the current stream: the union batch's row-gradient plan from the gathered CSR."""
        from . import ops
        W, B = self.world, self.B
        rp = self.rp_u.view(W, B + 1)
        rp.copy_(self.recv_csr[:, :B + 1].view(torch.int32))
        rp.add_(self.base_csr)
        flat = self.recv_csr.reshape(-1)
        self._union = ops.Csr(self.rp_u, flat.view(torch.int32), flat[self.cap:], self.n_items, rows=self.rows_u,
                              nb=W * B)
        ops.w1_rowgrad_plan(self._union, self.merged)

    def merge_apply(self, g_small: torch.Tensor):
        """Device-only: dense gradients <- rank-order sum of the weighted small gradients; the union row
        gradient <- the apply over the gathered da (after merge_plan)."""
        from . import ops
        torch.sum(self.recv_g, dim=0, out=g_small.reshape(-1))
        ops.w1_rowgrad_apply(self.recv_da, self.merged)
        return self.merged

    def unpack_merge(self, g_small: torch.Tensor):
        """Device-only (graph-capturable): dense gradients <- rank-order sum of the weighted packets; the union
        batch's first-layer row gradient <- the row-gradient kernels over the gathered (x, da)."""
        W, B, ns = self.world, self.B, self.ns
        torch.sum(self.recv[:, :ns], dim=0, out=g_small.reshape(-1))
        rp = self.rp_u.view(W, B + 1)
        rp.copy_(self.recv[:, self.off_rp:self.off_rp + B + 1].view(torch.int32))
        rp.add_(self.base)
        flat = self.recv.reshape(-1)
        if self.merge_fn is not _hip_merge and hasattr(self.merged, "rows_from_elsewhere"):
            self.merged.rows_from_elsewhere()  # no rowsq from an injected merge: the clip reads the rows
        self.merge_fn(self, self.rp_u, flat.view(torch.int32), flat[self.cap:], self.rows_u, W * B, self.recv_da,
                      self.merged)
        return self.merged


def _hip_make_merged(n_items, H, cap, device):
    from . import ops
    return ops.RowGradBuffers(n_items, H, cap, device)


def _hip_pack(ex: DPExchange, x, weight, rp_out, col_out, val_out, cap):
    from ._lib import check, lib, ptr
    check(lib().hvae_csr_batch_pack(x, float(weight), ptr(rp_out), ptr(col_out), ptr(val_out), cap,
                                    ptr(ex.overflow), torch.cuda.current_stream(ex.device).cuda_stream),
          "hvae_csr_batch_pack")


def _hip_merge(ex: DPExchange, row_ptr, col_idx, vals, rows, nb, da, out):
    """hvae_w1_rowgrad over the union batch: rows rank-major, each rank's rows in its batch order."""
    from . import ops
    ops.w1_rowgrad(ops.Csr(row_ptr, col_idx, vals, ex.n_items, rows=rows, nb=nb), da, out)
