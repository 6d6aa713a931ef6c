"""Fused, graph-captured HybridVAE train/validation step on MI355X.

Replaces the body of VAETrainer.train_epoch / validate (src/ml/train.py:81-124):
per batch the reference densifies every user row on the host, copies a dense
[B, N] batch to the device, runs ~60 eager aten ops through autograd, clips
with clip_grad_norm_, steps torch.optim.Adam and syncs three times with
.item(). Here one step is a fixed sequence of ~30 libhvae launches over
device-resident data, captured once per batch size into a hipGraph (through
torch.cuda.CUDAGraph) and replayed:

  * the interaction CSR lives in HBM; a batch is a window of a permuted
    user-id array whose start is a device counter (rows_offset), advanced by
    the graph itself -- no host work per step besides the replay;
  * parameters, gradients and Adam moments live in flat fp32 buffers; the
    module's nn.Parameters are rebound to views of the flat parameter buffer,
    so state_dict() and checkpoints always see the current values;
  * the first-layer weight is stored item-major (W1t [N, H]) -- the
    ``encoder.0.weight`` parameter is its [H, N] transposed view -- and its
    gradient is row-sparse (only the batch's items);
  * dropout masks and reparameterisation noise are Philox streams keyed by
    (seed, device step counter), so replays draw fresh randomness;
  * losses accumulate on the device in fp64 and are read once per epoch.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib, ops
from ._lib import CsrBatch, Epilogue, GemmDesc, check, lib, ptr

ALIGN = 4  # floats: every flat segment starts 16-B aligned


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class Seg:
    name: str
    offset: int
    shape: tuple
    numel: int


class FlatLayout:
    """Parameter layout: W1t [N, H1] first, then the small parameters.

    Small parameters keep the reference's parameter order (src/ml/model.py
    modules() order) except that fc_mu/fc_logvar weights (and biases) are
    adjacent, so that the two heads run as one [2L, H] GEMM.
    """

    def __init__(self, model):
        self.n_items = model.n_items
        self.hidden = list(model.hidden_dims)
        self.L = model.latent_dim
        self.d = model.embedding_dim
        self.has_proj = self.L != self.d
        segs: list[Seg] = []
        off = 0

        def add(name, shape, align=True):
            nonlocal off
            n = int(np.prod(shape))
            segs.append(Seg(name, off, tuple(shape), n))
            off = off + (_align(n) if align else n)

        add("w1t", (self.n_items, self.hidden[0]))
        self.small_offset = off
        # trainable item embeddings (HybridVAE(freeze_embeddings=False), reference model.py:72-75): E is the
        # reference's first parameter and has a dense gradient, so it opens the dense segment (clip + Adam cover it)
        self.train_e = bool(getattr(model, "item_embeddings_trainable", False))
        if self.train_e:
            add("item_embeddings", (self.n_items, self.d))
        prev = self.hidden[0]
        for k, hd in enumerate(self.hidden):
            i = 4 * k
            if k > 0:
                add(f"encoder.{i}.weight", (hd, prev))
            add(f"encoder.{i}.bias", (hd,))
            add(f"encoder.{i + 1}.weight", (hd,))
            add(f"encoder.{i + 1}.bias", (hd,))
            prev = hd
        add("fc_mu.weight", (self.L, prev), align=False)
        add("fc_logvar.weight", (self.L, prev))
        add("fc_mu.bias", (self.L,), align=False)
        add("fc_logvar.bias", (self.L,))
        if self.has_proj:
            add("projection_layer.0.weight", (self.d, self.L))
            add("projection_layer.0.bias", (self.d,))
            add("projection_layer.3.weight", (self.d, self.d))
            add("projection_layer.3.bias", (self.d,))
        self.total = off
        self.n_small = off - self.small_offset
        self.segs = {s.name: s for s in segs}

    def view(self, buf: torch.Tensor, name: str, base: int = 0) -> torch.Tensor:
        s = self.segs[name]
        return buf[s.offset - base: s.offset - base + s.numel].view(s.shape)

    def heads(self, buf: torch.Tensor, base: int = 0):
        """(W_heads [2L, H], b_heads [2L]) views spanning fc_mu and fc_logvar."""
        w, b = self.segs["fc_mu.weight"], self.segs["fc_mu.bias"]
        H = w.shape[1]
        W = buf[w.offset - base: w.offset - base + 2 * self.L * H].view(2 * self.L, H)
        B = buf[b.offset - base: b.offset - base + 2 * self.L]
        return W, B


@dataclass
class DeviceData:
    """Interaction CSR resident in HBM + the user ids a loader iterates over."""
    row_ptr: torch.Tensor
    col_idx: torch.Tensor
    vals: torch.Tensor
    users: torch.Tensor       # int32 [n] (rows of the matrix this dataset yields)
    n_items: int
    row_nnz: np.ndarray       # host copy of nnz per listed user (capacity planning)
    perm: torch.Tensor = field(default=None)  # int32 [n] current epoch order
    host_indptr: np.ndarray = field(default=None)   # host CSR (data-parallel exchange sizing)
    host_indices: np.ndarray = field(default=None)
    users_host: np.ndarray = field(default=None)
    dp_global: bool = False   # data parallel: every rank holds every user (hvae/dist.py dp_shard)
    _cap_cache: dict = field(default_factory=dict, repr=False)  # max_batch_nnz per batch size

    @staticmethod
    def from_scipy(mat, users, device) -> "DeviceData":
        mat = mat.tocsr()
        mat.sum_duplicates()
        users = np.asarray(users, dtype=np.int64)
        rp = mat.indptr.astype(np.int64)
        users_d = torch.as_tensor(users.astype(np.int32), device=device)
        return DeviceData(
            row_ptr=torch.as_tensor(rp, device=device),
            col_idx=torch.as_tensor(mat.indices.astype(np.int32), device=device),
            vals=torch.as_tensor(mat.data.astype(np.float32), device=device),
            users=users_d,
            n_items=mat.shape[1],
            row_nnz=(rp[users + 1] - rp[users]) if len(users) else np.zeros(0, np.int64),
            perm=users_d.clone(),  # fixed address: captured graphs read the epoch order from here
            host_indptr=rp, host_indices=mat.indices, users_host=users,
        )

    def max_batch_nnz(self, B: int) -> int:
        """Entries of the largest batch of B users (the sum of the B largest row lengths). Cached per B: the run
        loop asks once per step, and a sort of a million row lengths on the host (~1-4 ms) outlasted the Syn-1M
        step's GPU work, leaving the device idle between graph replays (~105 us a step, r06 kernel trace)."""
        if len(self.row_nnz) == 0:
            return 1
        hit = self._cap_cache.get(B)
        if hit is None:
            k = min(B, len(self.row_nnz))
            top = np.partition(self.row_nnz, len(self.row_nnz) - k)[len(self.row_nnz) - k:]
            hit = self._cap_cache[B] = max(int(top.sum()), 1)
        return hit


def _sampler_order(n: int, generator: torch.Generator | None, device) -> torch.Tensor:
    """The order DataLoader(shuffle=True) draws (torch RandomSampler.__iter__): with no generator, a fresh CPU
    generator seeded from the global RNG; with a CPU generator, randperm from it and a second draw the sampler
    makes when its iterator finishes; a device generator (benchmarks) draws on the device."""
    if generator is None:
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.randperm(n, generator=g)
    if generator.device.type != "cpu":
        return torch.randperm(n, generator=generator, device=generator.device)
    order = torch.randperm(n, generator=generator)
    torch.randperm(n, generator=generator)  # RandomSampler's trailing (empty-slice) draw
    return order


class _StepBuffers:
    """Activations / gradients for one batch size (graph-static pointers).

    cap: entries of the batch's first-layer row gradient (single GPU); with data parallelism the union
    batch's (world x the per-rank packet cap), which the clip workspace must cover."""

    def __init__(self, ex: "FusedTrainer", B: int, cap: int, train: bool):
        dev, lay = ex.device, ex.layout
        f = lambda *s: torch.empty(*s, device=dev)
        self.B = B
        H = lay.hidden
        L, d = lay.L, lay.d
        self.h = [f(B, hd) for hd in H]
        self.xhat = [f(B, hd) for hd in H]
        self.rstd = [f(B) for _ in H]
        self.a = [None] + [f(B, hd) for hd in H[1:]]
        self.heads = f(B, 2 * L)
        self.z = f(B, L)
        self.eps = f(B, L)
        self.kl_rows = f(B)
        self.p1 = f(B, d) if lay.has_proj else None
        self.q = f(B, d) if lay.has_proj else None
        self.u = f(B, d) if lay.has_proj else self.z
        self.lse = f(B)
        self.recon_rows = f(B)
        self.dU = f(B, d)
        self.dp1 = f(B, d) if lay.has_proj else None
        self.dz = f(B, L) if lay.has_proj else self.dU
        self.dheads = f(B, 2 * L)
        self.dh = [f(B, hd) for hd in H]
        self.da = [f(B, hd) for hd in H]
        self.loss3 = f(3)
        # the local row gradient (single GPU); data parallel steps build the union's in the exchange
        # (with trainable E the plan also gathers rows of u, width d)
        self.rg = (ops.RowGradBuffers(lay.n_items, H[0], cap, dev, width=d if ex.train_e else None)
                   if (train and ex.dp is None) else None)
        self.cap = cap
        # trainable E: dE's dense term in item chunks of e_chunk columns (S = u E_c^T, at most 64 M floats)
        self.e_chunk = 0
        if train and ex.train_e:
            self.e_chunk = int(min(lay.n_items, max(64, (1 << 26) // max(B, 1) // 64 * 64)))
            self.S = f(B, self.e_chunk)
            self.nrow = f(B)
        L_ = lib()
        need = [
            L_.hvae_decoder_workspace(ex.dec_dtype, B, lay.n_items, d),
            L_.hvae_clip_grad_norm_workspace(lay.n_small, cap, H[0]),
        ]
        dims = [(B, hd) for hd in H] + [(B, 2 * L), (B, d), (B, L)]
        for (_, n) in dims:
            need.append(L_.hvae_colsum_workspace(B, n))
        for hd in H:
            need.append(L_.hvae_ln_gelu_drop_bwd_workspace(B, hd))
        if B <= _lib.MLP_ROWS_MAX_NB:  # the row-parallel MLP backward's LayerNorm column sums
            need.append(L_.hvae_mlp_bwd_rows_workspace(B, H[-1]))
        # (m, n, k) of every split-K-capable GEMM of the step: forward, data- and weight-gradient products
        gemms = [(B, 2 * L, H[-1]), (2 * L, H[-1], B), (B, H[-1], 2 * L)]
        if lay.has_proj:
            gemms += [(B, d, L), (B, d, d), (d, d, B), (d, L, B), (B, d, d), (B, L, d)]
        for k in range(1, len(H)):
            gemms += [(B, H[k], H[k - 1]), (H[k], H[k - 1], B), (B, H[k - 1], H[k])]
        if self.e_chunk:
            gemms += [(B, self.e_chunk, d), (self.e_chunk, d, B)]
        for (m_, n_, k_) in gemms:
            need.append(L_.hvae_gemm_f32_workspace(m_, n_, k_))
        self.ws = torch.empty(max(int(max(need)), 256), dtype=torch.uint8, device=dev)
        # side-stream GEMMs: their split-K slabs must not alias the main stream's
        self.ws2 = torch.empty_like(self.ws) if ex.side is not None else None
        self.graph = None
        self.graph_k, self.graph_k_steps = None, 0  # single GPU: K consecutive steps in one graph (host-bound steps)
        self.graph_pre = self.graph_up = None  # data parallel: the CSR-packet and update graphs of a step
        self.graph_data = None  # the DeviceData a captured graph reads (held, compared by identity)


class FusedTrainer:
    """Owns the flat parameter/optimizer state of one HybridVAE on one device."""

    def __init__(self, model, device, lr: float = 1e-3, weight_decay: float = 0.0, betas=(0.9, 0.999),
                 eps: float = 1e-8, max_norm: float = 5.0, precision: str | None = None, seed: int | None = None,
                 use_graphs: bool = True, process_group=None):
        if device.type != "cuda":
            raise RuntimeError("FusedTrainer runs the MI355X HIP path only (device must be the HIP device)")
        lib()  # fail loudly now if libhvae.so is missing
        self.model = model
        self.device = device
        self.layout = lay = FlatLayout(model)
        self.lr, self.wd, self.betas, self.eps, self.max_norm = lr, weight_decay, betas, eps, max_norm
        self.use_graphs = use_graphs
        # trainable item embeddings: E lives in the flat dense segment; each step refreshes the decoder's image of
        # it, adds its gradient (hvae_embed.hip) and Adam moves it with the other dense parameters
        self.train_e = lay.train_e
        if self.train_e and process_group is not None and torch.distributed.get_world_size(process_group) > 1:
            raise NotImplementedError("fused trainer: data parallelism covers frozen item embeddings only (a "
                                      "trainable E would need its dense [N, d] gradient all-reduced every step)")
        self.seed = int(seed if seed is not None else torch.randint(0, 2 ** 62, (1,)).item())
        # ---- flat state
        self.flat = torch.zeros(lay.total, device=device)
        self.m = torch.zeros(lay.total, device=device)
        self.v = torch.zeros(lay.total, device=device)
        self.g_small = torch.zeros(lay.n_small, device=device)
        self._adopt_parameters()
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=device)
        self.step_snap = torch.zeros(1, dtype=torch.int64, device=device)  # step before this update (Adam's t - 1)
        # Exact lazy Adam for W1t (hvae_adam_lazy): rows outside a batch replay their g = 0 steps when next
        # read -- bitwise equal to torch's every-row update, without streaming all N*H each step.
        self.lazy_adam = not bool(int(os.environ.get("HVAE_DENSE_ADAM", "0")))
        self.last_step = torch.zeros(lay.n_items, dtype=torch.int32, device=device)
        self.tab_len = 1 << 22
        self.adam_tab = torch.zeros(2 * self.tab_len, dtype=torch.float32, device=device)
        # Deferred W1t update (hvae_adam_lazy_defer, HVAE_ADAM_DEFER=1): a step's update records its gradient rows
        # as pending instead of moving them; the next step's catch-up applies it to its batch's rows before the
        # forward reads them, and hvae_adam_lazy_pending moves the rest (and the step's sweep range) on the defer
        # stream beside the next step, joined before that step's row-gradient apply. Bitwise the same parameters.
        # HVAE_DEFER_AT: "sweep" (after the decoder sweep, beside the finalize and the backward) or "fwd" (forked
        # after the catch-up, beside the forward). It pays where few of a step's rows recur in the next batch: the
        # Syn-10M shard (N = 1 M, ~20 % recur) bf16 / fp8 -0.2..-0.4 % / -0.5..-1.2 % per step with "sweep" in 3 A/B
        # pairs each, "fwd" +-0.2 %; at Syn-1M (N = 100 K, ~48 % recur) the catch-up takes on half the rows' updates
        # and the rest slows the encoder beside it: 1.051 -> 1.081 ("sweep") / 1.096 ("fwd") ms; at the W = 8 union
        # (emulated, scripts/bench_dp_emul.py) the update graph's 0.96 ms moves into the next step's whole
        # (12.32 -> 12.30 bf16, 7.32 -> 7.29 fp8 ms): profiles/r06_defer_ab.jsonl. So HVAE_ADAM_DEFER defaults to
        # on from 2^19 items (HVAE_ADAM_DEFER=0 / 1 forces it)
        env_defer = os.environ.get("HVAE_ADAM_DEFER")
        self.adam_defer = self.lazy_adam and (bool(int(env_defer)) if env_defer is not None
                                              else lay.n_items >= (1 << 19))
        self.defer_at = os.environ.get("HVAE_DEFER_AT", "sweep")
        self._pend_open = False  # (host-tracked) a recorded update may still be pending on the device
        if self.adam_defer:
            self.pend_slot = torch.zeros(lay.n_items, dtype=torch.int32, device=device)
            self.pend_item = torch.zeros(lay.n_items, dtype=torch.int32, device=device)
            self.pend_hdr = torch.zeros(4, dtype=torch.int64, device=device)  # PendHdr (t = 0: nothing recorded)
            self._pend = _lib.AdamPend(ptr(self.pend_slot), ptr(self.pend_item), ptr(self.pend_hdr))
            self.defer_stream = torch.cuda.Stream(device)
        # A second stream for the optimizer-only work measured slower on MI355X: every cross-stream
        # edge of the captured graph costs 5-10 us, more than the short kernels it overlaps. Off by
        # default; the dependency structure stays in place for the larger configurations.
        self.two_streams = bool(int(os.environ.get("HVAE_TWO_STREAMS", "0")))
        # the weight-gradient GEMMs of the backward run on a second stream beside the data-gradient chain (batches
        # from plan_side_min_batch up; the plan keeps its own stream): Syn-1M 1.082 -> 1.061 ms per step, Syn-10M
        # bf16 / fp8 -0.1 / -0.3 % (profiles/r06_wgrad_side_ab.jsonl). HVAE_WGRAD_SIDE=0: one stream
        self.wgrad_side = bool(int(os.environ.get("HVAE_WGRAD_SIDE", "1")))
        self.side = torch.cuda.Stream(device) if (self.two_streams or self.wgrad_side) else None
        # the W1-gradient plan needs only the batch: it runs on its own stream beside the forward and is joined
        # before the row-gradient apply (the lazy-Adam catch-up then reads the batch's rows from the CSR)
        self.plan_side = bool(int(os.environ.get("HVAE_PLAN_SIDE", "1")))
        self.plan_stream = torch.cuda.Stream(device) if (self.plan_side and not self.two_streams) else None
        # below this batch the plan is short and the CSR catch-up's dependent loads cost more than the overlap
        # saves (All_Beauty B = 64: 0.1815 ms/step with the plan in line, 0.1965 beside; Syn-1M B = 4096:
        # 1.545 -> 1.293 ms/step beside)
        self.plan_side_min_batch = int(os.environ.get("HVAE_PLAN_SIDE_MIN_BATCH", "512"))
        # where the main stream joins the plan: "apply" (before the row-gradient apply, the plan overlapping the
        # catch-up, encoder and forward GEMMs) or "fwd" (before the first forward GEMM: the plan overlaps only the
        # catch-up and the encoder, and the forward GEMMs get every CU)
        self.plan_join = os.environ.get("HVAE_PLAN_JOIN", "apply")
        # when the plan forks off the main stream: "early" (before the lazy-Adam catch-up, so it overlaps the
        # catch-up too) or "late" (after it). Syn-1M 1.197 -> 1.189 ms per step, Syn-10M 11.35-11.38 -> 11.35-11.37
        # (profiles/r06_step_ab.jsonl); steps per graph replay 8 instead of 1 at B = 4096 changed nothing there
        self.plan_fork = os.environ.get("HVAE_PLAN_FORK", "early")
        # batches up to MLP_ROWS_MAX_NB run the latent / projection MLP row-parallel (hvae_mlp_*_rows)
        self.mlp_rows = bool(int(os.environ.get("HVAE_MLP_ROWS", "1")))
        self._mlp_rows_cache: dict[int, bool] = {}
        # and, when the batch's row-gradient plan fits one block, that plan as one more block of the same launch
        self.plan_in_rows = bool(int(os.environ.get("HVAE_PLAN_IN_ROWS", "1")))
        # the row-parallel MLP backward's LayerNorm column sums finished by the weight-gradient launch
        # (HVAE_LN_COLS_DEFERRED=0: in the backward launch, a last-block reduction)
        self.ln_cols_deferred = bool(int(os.environ.get("HVAE_LN_COLS_DEFERRED", "1")))
        # small batches: the fused encoder layer reads W1t through lazy Adam (HVAE_ENC_LAZY_READ=0: a catch-up launch)
        self.enc_lazy_read = bool(int(os.environ.get("HVAE_ENC_LAZY_READ", "1")))
        self.ones = torch.ones(1024, dtype=torch.float32, device=device)
        self.boff = torch.zeros(1, dtype=torch.int64, device=device)
        self.norm = torch.zeros(1, device=device)
        self.coef = torch.ones(1, device=device)
        self.accum_train = torch.zeros(3, dtype=torch.float64, device=device)
        # annealed beta (AnnealedVAE): the schedule's step counter and (beta, beta / B) of the current step, both
        # on the device, so an annealed epoch replays one captured step (hvae_anneal_beta)
        self.anneal_dev = torch.zeros(1, dtype=torch.int64, device=device)
        self.beta_dev = torch.zeros(2, device=device)
        self._anneal = None  # (beta_min, beta_max, anneal_steps) while an annealed train epoch runs
        self.accum_val = torch.zeros(3, dtype=torch.float64, device=device)
        self.host_step = 0
        # ---- frozen embeddings: fp32 (sparse terms, eval) + bf16 copy (decoder MFMA)
        self.E32 = model.item_embeddings.detach().contiguous()
        if self.E32.device != device:
            raise RuntimeError("model must be moved to the device before building the trainer")
        d = lay.d
        if precision is None:
            precision = "bf16" if ops.decoder_supported(_lib.HVAE_BF16, d) else "fp32"
        if precision == "bf16":
            if not ops.decoder_supported(_lib.HVAE_BF16, d):
                raise NotImplementedError(f"no bf16 streaming decoder for embedding dim {d}")
            self.dec_dtype = _lib.HVAE_BF16
            self.E_dec = ops.decoder_image(self.E32)  # bf16 E + its tile-transposed copy
        elif precision == "fp8":
            if not ops.decoder_supported(_lib.HVAE_FP8, d):
                raise NotImplementedError(f"no fp8 streaming decoder for embedding dim {d}")
            self.dec_dtype = _lib.HVAE_FP8
            self.E_dec = ops.decoder_image(self.E32, _lib.HVAE_FP8)  # bf16 E + e4m3 fragment tiles
        elif precision == "fp32":
            if not ops.decoder_supported(_lib.HVAE_F32, d):
                raise NotImplementedError(f"no fp32 streaming decoder for embedding dim {d}")
            self.dec_dtype = _lib.HVAE_F32
            self.E_dec = self.E32
        else:
            raise ValueError(f"precision must be 'bf16', 'fp8' or 'fp32', got {precision!r}")
        self.precision = precision
        self.enorm = ops.row_norm_max(self.E_dec)
        self._e_version = model.item_embeddings._version
        self._e_src_ptr = model.item_embeddings.data_ptr()
        self._bufs: dict[tuple, _StepBuffers] = {}
        self._views()
        self.dp = None
        self.dp_epoch = 0
        self.dp_val_epoch = 0
        self._dp_caps: dict = {}
        if process_group is not None and torch.distributed.get_world_size(process_group) > 1:
            from .dist import DPExchange
            self.dp = DPExchange(process_group, device, lay.n_items, lay.hidden[0], lay.n_small)
            # replicas start from rank 0's parameters (identical seeds make this a no-op, but be explicit)
            on_dev = torch.distributed.get_backend(process_group) == "nccl"
            flat = self.flat if on_dev else self.flat.cpu()
            torch.distributed.broadcast(flat, 0, group=process_group)
            if flat is not self.flat:
                self.flat.copy_(flat)
            seed_t = torch.tensor([self.seed], dtype=torch.int64, device=device if on_dev else "cpu")
            torch.distributed.broadcast(seed_t, 0, group=process_group)
            # the epoch order is drawn from rank 0's seed on every rank (dp_shard); per-rank dropout streams must
            # differ (each rank sees different users)
            self.dp_seed = int(seed_t.item())
            self.seed = self.dp_seed + 7919 * torch.distributed.get_rank(process_group)

    # ------------------------------------------------------------ state ---
    def _adopt_parameters(self):
        """Copy the module's parameters into the flat buffer and rebind them as views."""
        lay, model = self.layout, self.model
        named = dict(model.named_parameters())
        with torch.no_grad():
            w1 = named["encoder.0.weight"]  # [H, N] (a view of item-major storage)
            w1t = lay.view(self.flat, "w1t")
            w1t.copy_(w1.detach().t())
            w1.data = w1t.t()
            for name, seg in lay.segs.items():
                if name == "w1t":
                    continue
                p = named[name]
                v = lay.view(self.flat, name)
                v.copy_(p.detach().reshape(seg.shape))
                p.data = v
        self.param_views = {n: p for n, p in named.items()}

    def _views(self):
        lay, f = self.layout, self.flat
        base = lay.small_offset
        V = lambda buf, n, b=0: lay.view(buf, n, b)
        self.w1t = V(f, "w1t")
        self.m_w1t, self.v_w1t = V(self.m, "w1t"), V(self.v, "w1t")
        self.small = f[base:]
        self.m_small, self.v_small = self.m[base:], self.v[base:]
        H = lay.hidden
        self.P = {}
        self.G = {}
        for k in range(len(H)):
            i = 4 * k
            names = [f"encoder.{i}.bias", f"encoder.{i + 1}.weight", f"encoder.{i + 1}.bias"]
            if k > 0:
                names.append(f"encoder.{i}.weight")
            for n in names:
                self.P[n] = V(f, n)
                self.G[n] = V(self.g_small, n, base)
        if lay.train_e:
            self.P["item_embeddings"] = V(f, "item_embeddings")
            self.G["item_embeddings"] = V(self.g_small, "item_embeddings", base)
        self.W_heads, self.b_heads = lay.heads(f)
        self.gW_heads, self.gb_heads = lay.heads(self.g_small, base)
        if lay.has_proj:
            for n in ("projection_layer.0.weight", "projection_layer.0.bias", "projection_layer.3.weight",
                      "projection_layer.3.bias"):
                self.P[n] = V(f, n)
                self.G[n] = V(self.g_small, n, base)

    def sync_embeddings(self):
        """E is frozen, but load_state_dict / copy_ may still write new values into the module's buffer (a
        checkpoint of another embedding file): bring the fp32 copy, the decoder image and max||E|| up to date in
        place, so captured graphs keep their pointers. Cheap when nothing changed (a version compare)."""
        E = self.model.item_embeddings
        # the source tensor last synced from (its address and version), not E32's address: E32 is a private copy
        # whenever the module's buffer is non-contiguous or has been reassigned
        if E._version == self._e_version and E.data_ptr() == self._e_src_ptr:
            return
        with torch.no_grad():
            if E.data_ptr() != self.E32.data_ptr():
                self.E32.copy_(E.detach())
            if isinstance(self.E_dec, ops.DecoderImage):
                self.E_dec.refresh(self.E32)
            ops.row_norm_max(self.E_dec, out=self.enorm)
        self._e_version = E._version
        self._e_src_ptr = E.data_ptr()

    def grad_of(self, name: str) -> torch.Tensor:
        """Current gradient of a small parameter (after the last step)."""
        return self.G[name]

    # ------------------------------------------------------------- data ---
    def device_data(self, mat, users) -> DeviceData:
        return DeviceData.from_scipy(mat, users, self.device)

    # ------------------------------------------------------------- step ---
    def _buffers(self, B: int, cap: int, train: bool) -> _StepBuffers:
        key = (B, train)
        b = self._bufs.get(key)
        if b is None or (train and b.cap < cap):
            if b is not None:
                self._resolve_pending()  # a recorded update may still read the gradient rows of the set it replaces
            b = _StepBuffers(self, B, cap, train)
            self._bufs[key] = b
        return b

    def _csr(self, data: DeviceData, B: int, rows: torch.Tensor | None, offset: torch.Tensor | None) -> CsrBatch:
        return CsrBatch(ptr(data.row_ptr), ptr(data.col_idx), ptr(data.vals), ptr(rows), ptr(offset), B,
                        data.n_items)

    def _launch(self, bf: _StepBuffers, csr: CsrBatch, train: bool, beta: float, p_drop: float,
                ext: dict | None = None, advance: int = 0, weight: float = 1.0):
        """Enqueue one full step on the current stream (captured into a graph by the caller).

        advance > 0 also moves the device batch offset (rows_offset) by that many users. Data parallel:
        the batch CSR is exchanged before the forward (the union batch's row-gradient plan then runs beside
        it), the small gradients and da between the backward and the update; weight = this rank's share of the
        union batch.
        """
        if train and self.dp is not None:
            self._launch_pack_csr(bf, csr, weight)
            self.dp.communicate_csr()
            self._launch_fwd_bwd(bf, csr, train, beta, p_drop, ext)
            self._launch_pack_grads(bf, weight)
            self.dp.communicate_grads()
            self._launch_dp_update(bf, advance)
            return
        if train and not self._defers(bf.B) and not torch.cuda.is_current_stream_capturing():
            self._resolve_pending()  # this step's forward reads rows without the deferred update's catch-up
        self._launch_fwd_bwd(bf, csr, train, beta, p_drop, ext)
        if train:
            self._launch_update(bf.rg, bf, advance)
        elif advance:
            self._advance(advance)

    def _launch_pack_csr(self, bf: _StepBuffers | None, csr: CsrBatch | None, weight: float):
        """Start of a data-parallel step: this rank's batch as compact CSR (values * weight) into its packet.
        bf None: no users in this step."""
        if bf is None:
            self.dp.pack_csr(None, 0, 0.0)
            return
        self.dp.pack_csr(C.byref(csr), bf.B, weight)

    def _launch_pack_grads(self, bf: _StepBuffers | None, weight: float):
        """End of a data-parallel forward/backward: the weighted small gradients and the first-layer
        pre-activation gradient da."""
        if bf is None:
            self.dp.pack_grads(self.g_small.zero_(), 0, None, 0.0)
            return
        self.dp.pack_grads(self.g_small, bf.B, bf.da[0], weight)

    def _launch_dp_update(self, bf: _StepBuffers, advance: int):
        merged = self.dp.merge_apply(self.g_small)
        self._launch_update(merged, bf, advance)

    def _fork(self, src, dst):
        """dst waits for everything enqueued on src so far (a graph edge under capture)."""
        if src is dst:
            return
        ev = torch.cuda.Event()
        ev.record(src)
        dst.wait_event(ev)

    def _launch_fwd_bwd(self, bf: _StepBuffers, csr: CsrBatch, train: bool, beta: float, p_drop: float,
                        ext: dict | None = None):
        """Forward + loss (+ backward when train) of one batch.

        Two streams: the main stream runs the dependent chain (forward, decoder,
        data-gradient GEMMs, LayerNorm backward, W1 row gather); the side stream
        runs what only feeds the optimizer -- the W1 row-gradient plan (needs the
        batch only, so it overlaps the forward), the loss reduction and the
        weight-gradient GEMMs -- and is joined back before the update.
        """
        L_, lay = lib(), self.layout
        main = torch.cuda.current_stream(self.device)
        use_side = self.side is not None and (self.two_streams or bf.B >= self.plan_side_min_batch)
        side = self.side if use_side else main
        st, st2 = main.cuda_stream, side.cuda_stream
        B, H, Lt, d = bf.B, lay.hidden, lay.L, lay.d
        ws, wsn = ptr(bf.ws), bf.ws.numel()
        ws2 = ptr(bf.ws2) if side is not main else ws
        seed, step = self.seed, ptr(self.step_dev)
        tr = int(train)
        ext = ext or {}
        encm = ext.get("enc_masks", [None] * len(H))
        csr_ref = C.byref(csr)

        def gemm(ta, tb, M, N, K, A, lda, Bm, ldb, Cm, ldc, epi=None, beta_=0.0, rowsum=None, side_=False):
            if rowsum is not None:  # bias gradient = sum_k op(A)[m, k], fused into the weight-gradient GEMM
                epi = Epilogue(_lib.EPI_NONE, None, None, None, 0.0, None, 0, None, 0, 0, ptr(rowsum))
            check(L_.hvae_gemm_f32(ta, tb, M, N, K, 1.0, A, lda, Bm, ldb, beta_, Cm, ldc,
                                   C.byref(epi) if epi is not None else None, ws2 if side_ else ws, wsn,
                                   st2 if side_ else st), "gemm")

        ev_plan = None
        dp = self.dp is not None
        plan_in_rows = (train and not dp and not use_side and self.plan_in_rows and self._mlp_rows_ok(B)
                        and not (self.plan_stream is not None and B >= self.plan_side_min_batch)
                        and bf.rg.struct.cap <= _lib.PLAN_SMALL_CAP and B <= _lib.PLAN_SMALL_CAP)
        # one hidden layer of H <= 512 with the row-parallel MLP: the encoder layer runs in hvae_mlp_fwd_rows, which
        # can read W1t through lazy Adam itself (rows replayed in registers), so no catch-up launch precedes it
        fused_enc = self._mlp_rows_ok(B) and len(H) == 1 and H[0] <= 512
        enc_lazy = train and not dp and self.lazy_adam and self.enc_lazy_read and fused_enc
        # the last step's W1t update was recorded (hvae_adam_lazy_defer): the catch-up applies it to this batch's
        # rows, hvae_adam_lazy_pending to the rest on the defer stream
        defer = train and self._defers(B)
        ev_defer = None

        def launch_pending():
            nonlocal ev_defer
            ds = self.defer_stream
            self._fork(main, ds)
            cfg_p = ops.adam_config(self.lr, self.betas, self.eps, self.wd, self.step_dev, None)
            check(L_.hvae_adam_lazy_pending(C.byref(cfg_p), ptr(self.adam_tab), ptr(self.flat), ptr(self.m),
                                            ptr(self.v), ptr(self.last_step), lay.n_items, H[0],
                                            min(lay.n_items, bf.cap), C.byref(self._pend), ds.cuda_stream),
                  "adam_lazy_pending")
            ev_defer = torch.cuda.Event()
            ev_defer.record(ds)

        def catchup_csr():
            cfg0 = ops.adam_config(self.lr, self.betas, self.eps, self.wd, self.step_dev, None)
            if defer:
                check(L_.hvae_adam_lazy_catchup_csr_pending(
                    C.byref(cfg0), ptr(self.adam_tab), ptr(self.flat), ptr(self.m), ptr(self.v),
                    ptr(self.last_step), csr_ref, H[0], C.byref(self._pend), st), "adam_lazy_catchup_csr_pending")
            else:
                check(L_.hvae_adam_lazy_catchup_csr(C.byref(cfg0), ptr(self.adam_tab), ptr(self.flat), ptr(self.m),
                                                    ptr(self.v), ptr(self.last_step), csr_ref, H[0], st),
                      "adam_lazy_catchup_csr")
        if self.train_e:
            # E moved with the last step's Adam: the decoder's image of it and max||E|| follow (in the captured step)
            if isinstance(self.E_dec, ops.DecoderImage):
                self.E_dec.refresh(self.E32)
            ops.row_norm_max(self.E_dec, out=self.enorm)
        anneal = self._anneal if train else None
        beta_dev = None
        if anneal is not None:  # this step's (beta, beta / B) from the device schedule counter, which it advances
            beta_dev = self.beta_dev
            check(L_.hvae_anneal_beta(ptr(self.anneal_dev), anneal[0], anneal[1], anneal[2], B, ptr(beta_dev), st),
                  "anneal_beta")
        if train and dp:
            # data parallel: no local row gradient; the union batch's plan (from the CSR packets gathered
            # before this forward) runs on the plan stream beside it, its apply after the second exchange. The
            # batch's W1t rows replay their deferred steps, found from the CSR entries, before the forward
            # reads them
            if self.lazy_adam:
                catchup_csr()
            if defer and self.defer_at == "fwd":
                launch_pending()
            ps = self.plan_stream if self.plan_stream is not None else side
            if ps is not main:
                self._fork(main, ps)
                with torch.cuda.stream(ps):
                    self.dp.merge_plan()
                ev_plan = torch.cuda.Event()
                ev_plan.record(ps)
            else:
                self.dp.merge_plan()
        elif train and self.plan_stream is not None and B >= self.plan_side_min_batch:
            # the batch's W1t rows replay their deferred steps (found from the CSR) before the forward reads
            # them, while the row-gradient plan runs on the plan stream. With HVAE_PLAN_FORK=early the plan forks
            # before the catch-up (it reads only the batch, and the previous step's update that read the plan's
            # buffers is behind it on the main stream), so it overlaps the catch-up too
            ps = self.plan_stream
            early = self.plan_fork == "early"
            if early:
                self._fork(main, ps)
                check(L_.hvae_w1_rowgrad_plan(csr_ref, bf.rg.ref, ptr(bf.rg.ws), bf.rg.ws.numel(), ps.cuda_stream),
                      "w1_rowgrad_plan")
            if self.lazy_adam and not enc_lazy:
                catchup_csr()
            if defer and self.defer_at == "fwd":
                launch_pending()
            if not early:
                self._fork(main, ps)
                check(L_.hvae_w1_rowgrad_plan(csr_ref, bf.rg.ref, ptr(bf.rg.ws), bf.rg.ws.numel(), ps.cuda_stream),
                      "w1_rowgrad_plan")
            ev_plan = torch.cuda.Event()
            ev_plan.record(ps)
        elif train and plan_in_rows:
            # the plan runs as one more block of the row-parallel MLP forward's launch (hvae_mlp_fwd_rows); the
            # batch's W1t rows replay their deferred steps, found from the CSR, before the encoder reads them
            if self.lazy_adam and not enc_lazy:
                cfg0 = ops.adam_config(self.lr, self.betas, self.eps, self.wd, self.step_dev, None)
                check(L_.hvae_adam_lazy_catchup_csr(C.byref(cfg0), ptr(self.adam_tab), ptr(self.flat), ptr(self.m),
                                                    ptr(self.v), ptr(self.last_step), csr_ref, H[0], st),
                      "adam_lazy_catchup_csr")
        elif train:  # the row-gradient plan depends on the batch only: overlap it with the forward
            self._fork(main, side)
            check(L_.hvae_w1_rowgrad_plan(csr_ref, bf.rg.ref, ptr(bf.rg.ws), bf.rg.ws.numel(), st2),
                  "w1_rowgrad_plan")
            if self.lazy_adam and not enc_lazy:  # the batch's W1t rows replay their deferred steps before the forward
                cfg0 = ops.adam_config(self.lr, self.betas, self.eps, self.wd, self.step_dev, None)
                check(L_.hvae_adam_lazy_catchup(C.byref(cfg0), ptr(self.adam_tab), ptr(self.flat), ptr(self.m),
                                                ptr(self.v), ptr(self.last_step), bf.rg.ref, lay.n_items, H[0],
                                                st2), "adam_lazy_catchup")
                # the forward reads the rows this catch-up replays: it waits for it (HVAE_TWO_STREAMS=1 let the
                # encoder start beside it)
                self._fork(side, main)
            if side is not main:
                ev_plan = torch.cuda.Event()
                ev_plan.record(side)
        # ------------------------------------------------------ forward ---
        rows = self._mlp_rows_args(bf, B, tr, p_drop, ext, seed) if self._mlp_rows_ok(B) else None
        if rows is not None and len(H) == 1 and H[0] <= 512:
            # one hidden layer: the encoder layer runs in the row-parallel MLP forward's launch below
            rows.enc_x, rows.w1t, rows.b1 = C.pointer(csr), ptr(self.w1t), ptr(self.P["encoder.0.bias"])
            rows.ln_w, rows.ln_b = ptr(self.P["encoder.1.weight"]), ptr(self.P["encoder.1.bias"])
            rows.enc_drop_mult, rows.xhat, rows.rstd = ptr(encm[0]), ptr(bf.xhat[0]), ptr(bf.rstd[0])
            if enc_lazy:
                self._enc_adam = ops.adam_config(self.lr, self.betas, self.eps, self.wd, self.step_dev, None)
                rows.adam = C.addressof(self._enc_adam)
                rows.adam_m, rows.adam_v = ptr(self.m_w1t), ptr(self.v_w1t)
                rows.last_step, rows.adam_tab = ptr(self.last_step), ptr(self.adam_tab)
        else:
            check(L_.hvae_encoder_fwd(csr_ref, ptr(self.w1t), ptr(self.P["encoder.0.bias"]),
                                      ptr(self.P["encoder.1.weight"]), ptr(self.P["encoder.1.bias"]), H[0], p_drop,
                                      ptr(encm[0]), seed, step, tr, ptr(bf.h[0]), ptr(bf.xhat[0]),
                                      ptr(bf.rstd[0]), st), "encoder_fwd")
        for k in range(1, len(H)):
            i = 4 * k
            W = self.P[f"encoder.{i}.weight"]
            epi = Epilogue(_lib.EPI_BIAS, ptr(self.P[f"encoder.{i}.bias"]), None, None, 0.0, None, 0, None, 0, 0, None)
            gemm(0, 1, B, H[k], H[k - 1], ptr(bf.h[k - 1]), H[k - 1], ptr(W), H[k - 1], ptr(bf.a[k]), H[k], epi)
            check(L_.hvae_ln_gelu_drop_fwd(ptr(bf.a[k]), ptr(self.P[f"encoder.{i + 1}.weight"]),
                                           ptr(self.P[f"encoder.{i + 1}.bias"]), B, H[k], p_drop, ptr(encm[k]), seed,
                                           step, k, tr, ptr(bf.h[k]), ptr(bf.xhat[k]), ptr(bf.rstd[k]), st),
                  "ln_gelu_drop_fwd")
        Hl = H[-1]
        mu, lv = bf.heads, bf.heads[:, Lt:]
        if ev_plan is not None and self.plan_join == "fwd" and not dp:
            main.wait_event(ev_plan)
            ev_plan = None
        if rows is not None:
            if plan_in_rows:
                rows.plan_x, rows.plan_rg = C.pointer(csr), C.pointer(bf.rg.struct)
            # heads -> reparameterisation -> projection, the rows of the batch spread over blocks: one launch
            check(L_.hvae_mlp_fwd_rows(C.byref(rows), st), "mlp_fwd_rows")
        else:
            epi_b = Epilogue(_lib.EPI_BIAS, ptr(self.b_heads), None, None, 0.0, None, 0, None, 0, 0, None)
            gemm(0, 1, B, 2 * Lt, Hl, ptr(bf.h[-1]), Hl, ptr(self.W_heads), Hl, ptr(bf.heads), 2 * Lt, epi_b)
            check(L_.hvae_reparam_kl_fwd(ptr(mu), ptr(lv), 2 * Lt, B, Lt, tr, ptr(ext.get("eps")), seed, step,
                                         ptr(bf.z), ptr(bf.eps), ptr(bf.kl_rows), st), "reparam_kl_fwd")
        if lay.has_proj and rows is None:
            Wa, ba = self.P["projection_layer.0.weight"], self.P["projection_layer.0.bias"]
            Wb, bb = self.P["projection_layer.3.weight"], self.P["projection_layer.3.bias"]
            epi1 = Epilogue(_lib.EPI_BIAS_GELU_DROP, ptr(ba), ptr(bf.p1), None, p_drop, ptr(ext.get("proj_mask")),
                            seed, step, _lib.TAG_PROJ_DROP, tr, None)
            gemm(0, 1, B, d, Lt, ptr(bf.z), Lt, ptr(Wa), Lt, ptr(bf.q), d, epi1)
            epi2 = Epilogue(_lib.EPI_BIAS, ptr(bb), None, None, 0.0, None, 0, None, 0, 0, None)
            gemm(0, 1, B, d, d, ptr(bf.q), d, ptr(Wb), d, ptr(bf.u), d, epi2)
        if ev_plan is not None and self.plan_join == "sweep" and not dp:
            # (HVAE_PLAN_JOIN=sweep: the plan's last kernels finish before the sweep takes every CU, instead of
            # waiting beside it)
            main.wait_event(ev_plan)
            ev_plan = None
        accum = self.accum_train if train else self.accum_val
        # decoder sweep + finalize (split merge, sparse loss terms, du) + the batch loss means, one call
        check(L_.hvae_decoder_train(self.dec_dtype, ptr(bf.u), d, ptr(self.E_dec), ptr(self.enorm), ptr(self.E32),
                                    csr_ref, d, 1.0 / B, ptr(bf.lse), None, ptr(bf.recon_rows),
                                    ptr(bf.dU) if train else None, ptr(bf.kl_rows), beta, ptr(beta_dev),
                                    ptr(bf.loss3), ptr(accum), ws, wsn, st), "decoder_train")
        if not train:
            return
        if defer and ev_defer is None:  # HVAE_DEFER_AT=sweep: beside the finalize and the backward
            launch_pending()
        # ----------------------------------------------------- backward ---
        G = self.G
        if self.train_e:
            # dE's dense term (1/B) sum_b n_b softmax(u_b E^T)_i u_b in item chunks: S = u E_c^T, S <- (n_b / B)
            # exp(S - lse_b), dE_c = S^T u (hvae_embed.hip; the sparse term follows the plan, below)
            gE = G["item_embeddings"]
            check(L_.hvae_csr_row_sums(csr_ref, ptr(bf.nrow), st), "csr_row_sums")
            Cc, N_ = bf.e_chunk, lay.n_items
            for c0 in range(0, N_, Cc):
                cn = min(Cc, N_ - c0)
                gemm(0, 1, B, cn, d, ptr(bf.u), d, ptr(self.E32) + 4 * c0 * d, d, ptr(bf.S), Cc)
                check(L_.hvae_softmax_weights(ptr(bf.S), Cc, B, cn, ptr(bf.lse), ptr(bf.nrow), 1.0 / B, st),
                      "softmax_weights")
                gemm(1, 0, cn, d, B, ptr(bf.S), Cc, ptr(bf.u), d, ptr(gE) + 4 * c0 * d, d)

        def layer_bwd(wgrad: tuple, wrowsum, xgrad: tuple, xepi=None):
            """A layer's weight gradient (trans_a GEMM on the side stream) and data gradient: with one stream,
            both in one launch (hvae_gemm_f32_pair) -- they read only finished inputs."""
            if side is not main:
                self._fork(main, side)
                gemm(1, 0, *wgrad, rowsum=wrowsum, side_=True)
                gemm(0, 0, *xgrad, epi=xepi)
                return
            we = (Epilogue(_lib.EPI_NONE, None, None, None, 0.0, None, 0, None, 0, 0, ptr(wrowsum))
                  if wrowsum is not None else None)

            def desc(ta, args, e):
                M, N, K, A, lda, Bm, ldb, Cm, ldc = args
                return GemmDesc(ta, 0, M, N, K, 1.0, A, lda, Bm, ldb, 0.0, Cm, ldc,
                                C.pointer(e) if e is not None else None, ws, wsn)
            dw, dx = desc(1, wgrad, we), desc(0, xgrad, xepi)
            check(L_.hvae_gemm_f32_pair(C.byref(dw), C.byref(dx), st), "gemm_pair")

        if rows is not None:
            # the data gradients dp1 -> dheads -> dh of every row in one launch, then the three weight gradients
            # (with their bias gradients) in one more
            rows.dU, rows.dp1, rows.dheads, rows.dh = ptr(bf.dU), ptr(bf.dp1), ptr(bf.dheads), ptr(bf.dh[-1])
            rows.ks = beta / B
            rows.ks_dev = ptr(beta_dev[1:]) if beta_dev is not None else None
            # with the last hidden layer's LayerNorm -> GELU -> Dropout backward (dh -> da) fused
            kl_ = len(H) - 1
            il = 4 * kl_
            rows.ln_w, rows.ln_b = ptr(self.P[f"encoder.{il + 1}.weight"]), ptr(self.P[f"encoder.{il + 1}.bias"])
            rows.xhat, rows.rstd, rows.enc_drop_mult = ptr(bf.xhat[kl_]), ptr(bf.rstd[kl_]), ptr(encm[kl_])
            rows.enc_layer = kl_
            ln_grads = (G[f"encoder.{il + 1}.weight"], G[f"encoder.{il + 1}.bias"], G[f"encoder.{il}.bias"])
            rows.da = ptr(bf.da[kl_])
            if self.ln_cols_deferred:
                # the LayerNorm column sums stop at per-block partials in ws; the weight-gradient launch below adds
                # them in block order (partials^T x ones), instead of an in-kernel cross-block hand-off
                rows.d_ln_w = rows.d_ln_b = rows.d_bias = None
            else:
                rows.d_ln_w, rows.d_ln_b, rows.d_bias = (ptr(g) for g in ln_grads)
            rows.ws, rows.ws_bytes = ws, wsn
            check(L_.hvae_mlp_bwd_rows(C.byref(rows), st), "mlp_bwd_rows")
            keep = []

            def wdesc(M, N, A, lda, Bm, ldb, Cm, ldc, rowsum, K=B):
                e = Epilogue(_lib.EPI_NONE, None, None, None, 0.0, None, 0, None, 0, 0, ptr(rowsum))
                keep.append(e)
                return GemmDesc(1, 0, M, N, K, 1.0, A, lda, Bm, ldb, 0.0, Cm, ldc, C.pointer(e), None, 0)
            dl = [wdesc(d, d, ptr(bf.dU), d, ptr(bf.q), d, ptr(G["projection_layer.3.weight"]), d,
                        G["projection_layer.3.bias"]),
                  wdesc(d, Lt, ptr(bf.dp1), d, ptr(bf.z), Lt, ptr(G["projection_layer.0.weight"]), Lt,
                        G["projection_layer.0.bias"]),
                  wdesc(2 * Lt, Hl, ptr(bf.dheads), 2 * Lt, ptr(bf.h[-1]), Hl, ptr(self.gW_heads), Hl, self.gb_heads)]
            if self.ln_cols_deferred:
                nblk = int(L_.hvae_mlp_rows_blocks(B))
                for kind, g in enumerate(ln_grads):  # column sums of the [blocks, 3, H] partials: partials^T ones
                    dl.append(GemmDesc(1, 0, Hl, 1, nblk, 1.0, ws + 4 * kind * Hl, 3 * Hl,
                                       ptr(self.ones), 1, 0.0, ptr(g), 1, None, None, 0))
            descs = (GemmDesc * len(dl))(*dl)
            # (on the plan stream beside the W1 row gather this ran slower: All_Beauty 0.147 vs 0.129 ms per step,
            # profiles/r04_wgrad_beside_ab.jsonl)
            check(L_.hvae_gemm_f32_multi(descs, len(dl), st), "gemm_multi")
        elif lay.has_proj:
            epi3 = Epilogue(_lib.EPI_GELU_DROP_BWD, None, None, ptr(bf.p1), p_drop, ptr(ext.get("proj_mask")), seed,
                            step, _lib.TAG_PROJ_DROP, tr, None)
            layer_bwd((d, d, B, ptr(bf.dU), d, ptr(bf.q), d, ptr(G["projection_layer.3.weight"]), d),
                      G["projection_layer.3.bias"], (B, d, d, ptr(bf.dU), d, ptr(Wb), d, ptr(bf.dp1), d), epi3)
            # dz = dp1 Wa with the reparameterisation + KL backward as its epilogue -> dheads = [dmu | dlogvar]
            epi_r = Epilogue(_lib.EPI_REPARAM_BWD, None, None, ptr(bf.heads), 0.0, None, 0, None, 0, tr, None,
                             ptr(bf.eps), beta / B, ptr(beta_dev[1:]) if beta_dev is not None else None)
            layer_bwd((d, Lt, B, ptr(bf.dp1), d, ptr(bf.z), Lt, ptr(G["projection_layer.0.weight"]), Lt),
                      G["projection_layer.0.bias"], (B, Lt, d, ptr(bf.dp1), d, ptr(Wa), Lt, ptr(bf.dheads), 2 * Lt),
                      epi_r)
        else:
            dmu, dlv = bf.dheads, bf.dheads[:, Lt:]
            check(L_.hvae_reparam_kl_bwd(ptr(bf.dz), ptr(mu), ptr(lv), 2 * Lt, ptr(bf.eps), B, Lt, beta / B,
                                         ptr(beta_dev[1:]) if beta_dev is not None else None, tr,
                                         ptr(dmu), ptr(dlv), 2 * Lt, st), "reparam_kl_bwd")
        if rows is None:
            layer_bwd((2 * Lt, Hl, B, ptr(bf.dheads), 2 * Lt, ptr(bf.h[-1]), Hl, ptr(self.gW_heads), Hl),
                      self.gb_heads, (B, Hl, 2 * Lt, ptr(bf.dheads), 2 * Lt, ptr(self.W_heads), Hl, ptr(bf.dh[-1]), Hl))
        for k in range(len(H) - 1, -1, -1):
            i = 4 * k
            if not (rows is not None and k == len(H) - 1):  # (the row-parallel MLP backward did the last one)
                check(L_.hvae_ln_gelu_drop_bwd(
                    ptr(bf.dh[k]), ptr(bf.xhat[k]), ptr(bf.rstd[k]), ptr(self.P[f"encoder.{i + 1}.weight"]),
                    ptr(self.P[f"encoder.{i + 1}.bias"]), B, H[k], p_drop, ptr(encm[k]), seed, step, k, tr,
                    ptr(bf.da[k]), ptr(G[f"encoder.{i + 1}.weight"]), ptr(G[f"encoder.{i + 1}.bias"]),
                    ptr(G[f"encoder.{i}.bias"]), ws, wsn, st), "ln_gelu_drop_bwd")
            if k > 0:
                W = self.P[f"encoder.{i}.weight"]
                layer_bwd((H[k], H[k - 1], B, ptr(bf.da[k]), H[k], ptr(bf.h[k - 1]), H[k - 1],
                           ptr(G[f"encoder.{i}.weight"]), H[k - 1]), None,
                          (B, H[k - 1], H[k], ptr(bf.da[k]), H[k], ptr(W), H[k - 1], ptr(bf.dh[k - 1]), H[k - 1]))
        if ev_plan is not None:
            main.wait_event(ev_plan)
        if ev_defer is not None:  # the recorded update's rows are done before this step's apply rewrites its rows
            main.wait_event(ev_defer)
        if not dp:
            if self.train_e:
                # dE's sparse term -(1/B) sum_b x_bi u_b over the plan's item segments (the apply with u for da),
                # before the W1 rows take the same buffer
                check(L_.hvae_w1_rowgrad_apply(ptr(bf.u), d, bf.rg.ref, st), "w1_rowgrad_apply(u)")
                check(L_.hvae_rowgrad_scatter_rows(bf.rg.ref, d, -1.0 / B, ptr(G["item_embeddings"]), d, st),
                      "rowgrad_scatter_rows")
            check(L_.hvae_w1_rowgrad_apply(ptr(bf.da[0]), H[0], bf.rg.ref, st), "w1_rowgrad_apply")
        self._fork(side, main)  # join: every gradient is complete on the main stream

    def _mlp_rows_ok(self, B: int) -> bool:
        """The row-parallel latent / projection MLP (hvae_mlp_fwd_rows / _bwd_rows) serves this batch:
        a projection layer, B <= MLP_ROWS_MAX_NB, widths that are multiples of 32 up to 1024 whose
        activations fit the kernels' LDS. HVAE_MLP_ROWS=0 keeps the GEMM chain."""
        lay = self.layout
        if not self.mlp_rows or not lay.has_proj or B > _lib.MLP_ROWS_MAX_NB:
            return False
        ok = self._mlp_rows_cache.get(B)
        if ok is None:  # the library's own shape rules (rows per block, LDS of both directions), asked for the
            # configuration the step launches: the fused encoder layer (one hidden layer of at most 512) needs its
            # own LDS beside the MLP's
            fused_enc = int(len(lay.hidden) == 1 and lay.hidden[0] <= 512)
            ok = bool(lib().hvae_mlp_rows_supported(B, lay.hidden[-1], lay.L, lay.d, fused_enc))
            self._mlp_rows_cache[B] = ok
        return ok

    def _mlp_rows_args(self, bf: _StepBuffers, B: int, tr: int, p_drop: float, ext: dict, seed: int):
        lay = self.layout
        return _lib.MlpRows(
            nb=B, H=lay.hidden[-1], L=lay.L, D=lay.d,
            W_heads=ptr(self.W_heads), b_heads=ptr(self.b_heads),
            W_a=ptr(self.P["projection_layer.0.weight"]), b_a=ptr(self.P["projection_layer.0.bias"]),
            W_b=ptr(self.P["projection_layer.3.weight"]), b_b=ptr(self.P["projection_layer.3.bias"]),
            train=tr, p_drop=p_drop, drop_mult=ptr(ext.get("proj_mask")), eps_in=ptr(ext.get("eps")), seed=seed,
            step_dev=ptr(self.step_dev), h=ptr(bf.h[-1]), heads=ptr(bf.heads), z=ptr(bf.z), eps=ptr(bf.eps),
            kl_rows=ptr(bf.kl_rows), p1=ptr(bf.p1), q=ptr(bf.q), u=ptr(bf.u))

    def _launch_update(self, rg, bf: _StepBuffers, advance: int = 0):
        """clip_grad_norm_(5.0) + Adam over the flat state: two launches.

        The clip launch also advances the step counter (and the batch offset);
        Adam reads the pre-increment step from step_snap.
        """
        L_, lay = lib(), self.layout
        st = torch.cuda.current_stream(self.device).cuda_stream
        H = lay.hidden
        ws, wsn = ptr(bf.ws), bf.ws.numel()
        cfg = ops.adam_config(self.lr, self.betas, self.eps, self.wd, self.step_snap, self.coef)
        if self.lazy_adam:  # the clip's last block also writes the step's Adam scalars into the step table
            check(L_.hvae_clip_grad_norm_step_adam(ptr(self.g_small), lay.n_small, rg.ref, H[0], self.max_norm,
                                                   ptr(self.norm), ptr(self.coef), ptr(self.step_dev),
                                                   ptr(self.step_snap), ptr(self.boff) if advance else None, advance,
                                                   C.byref(cfg), ptr(self.adam_tab), ws, wsn, st),
                  "clip_grad_norm_step_adam")
        else:
            check(L_.hvae_clip_grad_norm_step(ptr(self.g_small), lay.n_small, rg.ref, H[0], self.max_norm,
                                              ptr(self.norm), ptr(self.coef), ptr(self.step_dev),
                                              ptr(self.step_snap), ptr(self.boff) if advance else None, advance,
                                              ws, wsn, st), "clip_grad_norm_step")
        # W1t (row-sparse gradient, offset 0 of the flat buffer) and the dense segment in one launch
        if self.lazy_adam and self._defers(bf.B):  # W1t's rows recorded, moved by the next step (or a flush)
            check(L_.hvae_adam_lazy_defer(C.byref(cfg), ptr(self.adam_tab), self.tab_len, ptr(self.flat),
                                          ptr(self.m), ptr(self.v), ptr(self.last_step), rg.ref, H[0],
                                          ptr(self.g_small), lay.small_offset, lay.n_small, C.byref(self._pend), st),
                  "adam_lazy_defer")
            self._pend_open = True
        elif self.lazy_adam:
            check(L_.hvae_adam_lazy(C.byref(cfg), ptr(self.adam_tab), self.tab_len, ptr(self.flat), ptr(self.m),
                                    ptr(self.v), ptr(self.last_step), rg.ref, H[0], ptr(self.g_small),
                                    lay.small_offset, lay.n_small, st), "adam_lazy")
        else:
            check(L_.hvae_adam_flat(C.byref(cfg), ptr(self.flat), ptr(self.m), ptr(self.v), rg.ref, lay.n_items,
                                    H[0], ptr(self.g_small), lay.small_offset, lay.n_small, st), "adam_flat")

    def flush(self):
        """Bring every W1t row (and its m, v) up to the completed step count (lazy Adam).

        Called at the end of every epoch and eager step, so that whatever reads the
        parameters or the optimizer state next sees torch's values.
        """
        if not self.lazy_adam:
            return
        self._resolve_pending()
        cfg0 = ops.adam_config(self.lr, self.betas, self.eps, self.wd, self.step_dev, None)
        check(lib().hvae_adam_lazy_catchup(C.byref(cfg0), ptr(self.adam_tab), ptr(self.flat), ptr(self.m),
                                           ptr(self.v), ptr(self.last_step), None, self.layout.n_items,
                                           self.layout.hidden[0], torch.cuda.current_stream(self.device).cuda_stream),
              "adam_lazy_flush")

    def _defers(self, B: int) -> bool:
        """Whether a train step of B users records its W1t update (hvae_adam_lazy_defer) instead of applying it:
        the steps whose forward is preceded by the CSR catch-up and whose plan runs on its own stream (data
        parallel, or B >= plan_side_min_batch), not the small batches whose fused encoder reads W1t through lazy
        Adam itself."""
        if not (self.adam_defer and self.lazy_adam) or self.two_streams:  # (lazy_adam may be switched off later)
            return False
        if self.dp is not None:
            return True
        if self.plan_stream is None or B < self.plan_side_min_batch:
            return False
        H = self.layout.hidden
        return not (self.enc_lazy_read and self._mlp_rows_ok(B) and len(H) == 1 and H[0] <= 512)

    def _resolve_pending(self):
        """Apply a recorded W1t update still pending, on the current stream (eager; a no-op on the device when
        the next step's catch-up and hvae_adam_lazy_pending already did)."""
        if not self._pend_open:
            return
        lay = self.layout
        cfg0 = ops.adam_config(self.lr, self.betas, self.eps, self.wd, self.step_dev, None)
        check(lib().hvae_adam_lazy_pending(C.byref(cfg0), ptr(self.adam_tab), ptr(self.flat), ptr(self.m),
                                           ptr(self.v), ptr(self.last_step), lay.n_items, lay.hidden[0],
                                           lay.n_items, C.byref(self._pend),
                                           torch.cuda.current_stream(self.device).cuda_stream), "adam_lazy_pending")
        self._pend_open = False

    def _hyper(self) -> tuple:
        """The optimizer constants a captured step bakes in (part of its graph key)."""
        return (self.lr, self.betas, self.eps, self.wd, self.max_norm)

    def mark_all_current(self):
        """Every row has had every step applied (after an external dense update of W1t)."""
        self._resolve_pending()
        self.last_step.copy_(self.step_dev.to(torch.int32).expand_as(self.last_step))

    def _check_steps(self, more: int):
        if self.lazy_adam and self.host_step + more + 2 >= self.tab_len:
            raise RuntimeError("lazy Adam step table exhausted; run with HVAE_DENSE_ADAM=1")

    def _advance(self, B: int):
        check(lib().hvae_counter_add(ptr(self.boff), B, torch.cuda.current_stream(self.device).cuda_stream),
              "counter_add")

    # -------------------------------------------------------- public API ---
    def step_batch(self, data: DeviceData, rows: torch.Tensor | None, B: int, beta: float, p_drop: float,
                   train: bool = True, ext: dict | None = None, weight: float | None = None) -> torch.Tensor:
        """One eager step over `rows` (int32 device user ids, or None: rows 0..B-1). Returns loss3.

        Data parallel (train): every rank calls it together with its own rows; weight = this rank's share of
        the union batch (default 1 / world: equal batches)."""
        self.sync_embeddings()
        cap = int(data.row_ptr[-1].item()) if rows is None else data.max_batch_nnz(B)
        dp = self.dp if train else None
        if dp is not None:
            cap = int(dp.all_reduce([cap], op=torch.distributed.ReduceOp.MAX)[0])
            dp.plan(B, cap)
            cap *= dp.world
        bf = self._buffers(B, cap, train)
        csr = self._csr(data, B, rows, None)
        if train:
            self._check_steps(1)
        else:
            self.flush()
        self._launch(bf, csr, train, beta, p_drop, ext,
                     weight=(1.0 / dp.world if weight is None else weight) if dp is not None else 1.0)
        if train:
            self.host_step += 1
            self.flush()
            if dp is not None:
                dp.check()
        return bf.loss3

    def run_epoch(self, data: DeviceData, batch_size: int, shuffle: bool, beta_fn, p_drop: float,
                  train: bool = True, drop_last: bool = False, generator: torch.Generator | None = None,
                  max_batches: int | None = None) -> dict:
        """Iterate the dataset in batches (DataLoader semantics: shuffle, drop_last=False).

        beta_fn(step_index) -> beta; a constant beta (ConstBeta) or the annealed schedule evaluated on the device
        (AnnealedBeta) lets every full batch replay one graph.
        Returns the mean of the per-batch losses (VAETrainer.train_epoch's metric).
        """
        n = int(data.users.numel())
        if n == 0:
            nan = {"total_loss": float("nan"), "recon_loss": float("nan"), "kl_loss": float("nan")}
            if not train and self.dp is not None and not data.dp_global:
                # an empty shard still joins the other ranks' batch-weighted validation sum
                tot = self.dp.all_reduce([0.0, 0.0, 0.0, 0.0]).tolist()
                if tot[3] > 0:
                    return {"total_loss": tot[0] / tot[3], "recon_loss": tot[1] / tot[3], "kl_loss": tot[2] / tot[3]}
            return nan
        self.sync_embeddings()
        anneal = getattr(beta_fn, "anneal", None) if train else None
        if anneal is not None:
            self.anneal_dev.fill_(int(beta_fn.model.current_step))
        self._anneal = anneal
        try:
            if train and self.dp is not None:
                out, steps = self._run_epoch_dp(data, batch_size, shuffle, beta_fn, p_drop, drop_last, generator,
                                                max_batches)
            else:
                out, steps = self._run_epoch_local(data, batch_size, shuffle, beta_fn, p_drop, train, drop_last,
                                                   generator, max_batches)
        finally:
            self._anneal = None
        if anneal is not None:  # the host mirror of the device schedule counter (AnnealedVAE.step_annealing)
            beta_fn.model.current_step += steps
        return out

    @staticmethod
    def _step_beta(beta_fn, const_beta, anneal, i: int):
        """The beta argument of step i: the constant, a placeholder when the device schedule supplies it, or
        beta_fn(i) (a host schedule: eager steps)."""
        if const_beta is not None:
            return const_beta
        return 0.0 if anneal is not None else beta_fn(i)

    def _run_epoch_local(self, data: DeviceData, batch_size: int, shuffle: bool, beta_fn, p_drop: float,
                         train: bool, drop_last: bool, generator, max_batches) -> tuple[dict, int]:
        n = int(data.users.numel())
        shard_reduce = False
        if not train and self.dp is not None and data.users_host is not None:
            if data.dp_global:  # every rank holds every user: deal the single-GPU batches over the ranks
                return self._run_eval_sharded(data, batch_size, shuffle, beta_fn, p_drop, drop_last, generator,
                                              max_batches)
            # per-rank shards: each rank validates its whole shard, then the batch losses are summed over ranks
            shard_reduce = True
        if shuffle:
            order = _sampler_order(n, generator, self.device)
            data.perm.copy_(data.users[order.to(self.device)])
        else:
            data.perm.copy_(data.users)
        accum = self.accum_train if train else self.accum_val
        accum.zero_()
        self.boff.zero_()
        if train:
            self._check_steps(n // batch_size + 1)
        else:
            self.flush()  # the forward reads W1t rows that no catch-up precedes
        n_full, tail = divmod(n, batch_size)
        if drop_last:
            tail = 0
        if max_batches is not None:  # bounded pass (benchmarks): full batches only
            n_full, tail = min(n_full, max_batches), 0
        n_batches = n_full + (1 if tail else 0)
        const_beta = getattr(beta_fn, "constant", None)
        anneal = self._anneal
        B = batch_size
        bi = 0
        while bi < n_full:
            beta = self._step_beta(beta_fn, const_beta, anneal, bi)
            bf = self._buffers(B, data.max_batch_nnz(B), train)
            if self.use_graphs and (const_beta is not None or anneal is not None):
                done = self._replay(bf, data, train, beta, p_drop, bi, (beta, anneal, p_drop) + self._hyper(),
                                    n_full - bi)
            else:
                self._launch(bf, self._csr(data, B, data.perm, self.boff), train, beta, p_drop, advance=B)
                done = 1
            if train:
                self.host_step += done
            bi += done
        if tail:
            beta = self._step_beta(beta_fn, const_beta, anneal, n_full)
            bf = self._buffers(tail, data.max_batch_nnz(tail), train)
            self._launch(bf, self._csr(data, tail, data.perm, self.boff), train, beta, p_drop, advance=tail)
            if train:
                self.host_step += 1
        self.flush()
        sums = accum.cpu().tolist()  # the one host sync of the epoch
        if shard_reduce:  # batch-weighted: the mean over every rank's batches, as one GPU over all shards
            tot = self.dp.all_reduce(np.array(sums + [float(n_batches)], dtype=np.float64)).tolist()
            sums, n_batches = tot[:3], int(round(tot[3]))
        return ({"total_loss": sums[0] / n_batches, "recon_loss": sums[1] / n_batches,
                 "kl_loss": sums[2] / n_batches}, n_batches if train else 0)

    def _run_eval_sharded(self, data: DeviceData, B: int, shuffle: bool, beta_fn, p_drop: float, drop_last: bool,
                          generator, max_batches) -> tuple[dict, int]:
        """Data-parallel validation (VAETrainer.validate under torchrun): the epoch's batches -- the ones a single
        GPU would form, in its order -- are dealt round-robin over the ranks (batch i to rank i mod W), each rank
        runs its own through the same captured eval step, and the per-batch loss sums are all-reduced. Every
        batch is the single-GPU batch, so the result is the single-GPU validation loss up to the order of the
        fp64 sum over batches."""
        dp, W, r = self.dp, self.dp.world, self.dp.rank
        users = data.users_host
        n = len(users)
        if shuffle:  # one order on every rank
            if generator is not None:
                # the caller's generator decides it, as in a single-GPU run: every rank draws the permutation
                # exactly as _sampler_order does (so each generator ends in the state a single-GPU validation
                # leaves it in) and rank 0's permutation is broadcast (so the ranks agree even if their generators
                # do not): the batches are the single-GPU batches
                grp = dp.group
                on_dev = torch.distributed.get_backend(grp) == "nccl"
                perm = _sampler_order(n, generator, self.device).to(torch.int64)
                perm = perm.to(self.device if on_dev else "cpu")
                torch.distributed.broadcast(perm, torch.distributed.get_global_rank(grp, 0), group=grp)
                order = users[perm.cpu().numpy()]
            else:  # the shared data-parallel seed
                rng = np.random.default_rng([self.dp_seed, 0x5EA1, self.dp_val_epoch])
                self.dp_val_epoch += 1
                order = users[rng.permutation(n)]
        else:
            order = users
        n_full, tail = divmod(n, B)
        if drop_last:
            tail = 0
        if max_batches is not None:
            n_full, tail = min(n_full, max_batches), 0
        n_batches = n_full + (1 if tail else 0)
        mine_full = list(range(r, n_full, W))
        mine_tail = bool(tail) and n_full % W == r
        parts = [order[i * B:(i + 1) * B] for i in mine_full] + ([order[n_full * B:n_full * B + tail]] if mine_tail
                                                                   else [])
        if parts:
            mine = np.concatenate(parts).astype(np.int32)
            data.perm[:len(mine)].copy_(torch.as_tensor(mine).to(self.device))
        self.accum_val.zero_()
        self.boff.zero_()
        self.flush()  # the forward reads W1t rows that no catch-up precedes
        const_beta = getattr(beta_fn, "constant", None)
        for k, bi in enumerate(mine_full):
            beta = const_beta if const_beta is not None else beta_fn(bi)
            bf = self._buffers(B, data.max_batch_nnz(B), False)
            if self.use_graphs and const_beta is not None:
                self._replay(bf, data, False, beta, p_drop, k, (beta, None, p_drop) + self._hyper())
            else:
                self._launch(bf, self._csr(data, B, data.perm, self.boff), False, beta, p_drop, advance=B)
        if mine_tail:
            beta = const_beta if const_beta is not None else beta_fn(n_full)
            bf = self._buffers(tail, data.max_batch_nnz(tail), False)
            self._launch(bf, self._csr(data, tail, data.perm, self.boff), False, beta, p_drop, advance=tail)
        tot = dp.all_reduce(self.accum_val.cpu().numpy()).tolist()  # the batches' losses summed over the ranks
        if n_batches == 0:
            return {"total_loss": float("nan"), "recon_loss": float("nan"), "kl_loss": float("nan")}, 0
        return {"total_loss": tot[0] / n_batches, "recon_loss": tot[1] / n_batches,
                "kl_loss": tot[2] / n_batches}, 0

    def _replay(self, bf: _StepBuffers, data: DeviceData, train: bool, beta: float, p_drop: float, bi: int,
                key, left: int = 1) -> int:
        """Run full batches through their captured graph(s), capturing them first if needed; returns the steps
        run. The first use of a buffer set runs one step eagerly instead (loads kernels, sets attributes). A graph
        holds the DeviceData it reads (compared by identity, so a freed dataset's address reused by a new one
        never replays a stale graph). Single GPU: where `left` allows, one replay of the K-step graph runs K
        consecutive steps (the batch offset advances on the device), so the host pays one replay per K steps."""
        if bf.graph is None or bf.graph_key != key or bf.graph_data is not data:
            if bi == 0 and bf.graph is None:
                self._launch(bf, self._csr(data, bf.B, data.perm, self.boff), train, beta, p_drop, advance=bf.B,
                             weight=key[-1] if self.dp is not None and train else 1.0)
                return 1
            self._capture(bf, data, train, beta, p_drop, key)
        defer = train and self._defers(bf.B)
        if train and not defer:
            self._resolve_pending()  # the graph's forward reads rows without the recorded update's catch-up
        if bf.graph_k is not None and left >= bf.graph_k_steps:
            bf.graph_k.replay()
            self._pend_open = self._pend_open or defer
            return bf.graph_k_steps
        if bf.graph_pre is not None:  # data parallel: the CSR packet, then its exchange
            bf.graph_pre.replay()
            self.dp.communicate_csr()
        bf.graph.replay()
        if bf.graph_up is not None:  # data parallel: the gradients' exchange between the step's graphs
            self.dp.communicate_grads()
            bf.graph_up.replay()
        self._pend_open = self._pend_open or defer
        return 1

    # ------------------------------------------------------ data parallel ---
    def _dp_cap(self, data: DeviceData, B: int) -> int:
        """Entries of the largest batch of B users any rank can draw (agreed once per dataset and B)."""
        key = (id(data), B)
        hit = self._dp_caps.get(key)
        if hit is None or hit[0] is not data:
            cap = int(self.dp.all_reduce([data.max_batch_nnz(B)], op=torch.distributed.ReduceOp.MAX)[0])
            self._dp_caps[key] = hit = (data, max(cap, 1))
        return hit[1]

    def _run_epoch_dp(self, data: DeviceData, B: int, shuffle: bool, beta_fn, p_drop: float, drop_last: bool,
                      generator, max_batches) -> tuple[dict, int]:
        """A data-parallel training epoch (hvae/dist.py). data.dp_global: every rank holds every user and takes
        its slice of each global batch of a permutation drawn from the shared seed; otherwise the ranks'
        datasets are their own shards, which must have equal sizes."""
        from .dist import dp_shard
        dp, W, r = self.dp, self.dp.world, self.dp.rank
        users = data.users_host
        n = len(users)
        if data.dp_global:
            rng = np.random.default_rng([self.dp_seed, self.dp_epoch])
            order = users[rng.permutation(n)] if shuffle else users
            mine, n_full, counts = dp_shard(order, B, W, r)
        else:
            sizes = dp.all_reduce([n, -n], op=torch.distributed.ReduceOp.MAX)
            if int(sizes[0]) != n or int(-sizes[1]) != n:
                raise ValueError("data-parallel shards of unequal sizes: give every rank the whole dataset "
                                 "(DeviceData.dp_global) or equal shards")
            # the rank's own shard in the sampler's order, gathered on the device (a host round trip of the
            # order and the users cost ~10-45 ms per epoch at 1.25 M users: scripts/bench_dp_emul.py)
            order = _sampler_order(n, generator, self.device) if shuffle else None
            mine = data.users[order.to(self.device)] if order is not None else data.users
            n_full, t = divmod(n, B)
            counts = [t] * W
        self.dp_epoch += 1
        if drop_last:
            counts = [0] * W
        if max_batches is not None:
            n_full, counts = min(n_full, max_batches), [0] * W
        if isinstance(mine, torch.Tensor):
            data.perm[:len(mine)].copy_(mine)
        else:
            data.perm[:len(mine)].copy_(torch.as_tensor(np.asarray(mine, dtype=np.int32)).to(self.device))
        self.accum_train.zero_()
        self.boff.zero_()
        n_steps = n_full + (1 if sum(counts) else 0)
        self._check_steps(n_steps + 1)
        const_beta = getattr(beta_fn, "constant", None)
        anneal = self._anneal
        cap = self._dp_cap(data, B)
        if n_full:
            dp.plan(B, cap)
        for bi in range(n_full):
            beta = self._step_beta(beta_fn, const_beta, anneal, bi)
            bf = self._buffers(B, W * cap, True)
            if self.use_graphs and (const_beta is not None or anneal is not None):
                self._replay(bf, data, True, beta, p_drop, bi, (beta, anneal, p_drop) + self._hyper() + (cap, 1.0 / W))
            else:
                self._launch(bf, self._csr(data, B, data.perm, self.boff), True, beta, p_drop, advance=B,
                             weight=1.0 / W)
            self.host_step += 1
        sums = self.accum_train.cpu().numpy() / W  # the union batch's loss = mean of equal shares
        if sum(counts):  # the last, partial global batch: eager, every rank takes part (possibly with no users)
            T, c, Bt = sum(counts), counts[r], max(counts)
            beta = self._step_beta(beta_fn, const_beta, anneal, n_full)
            dp.plan(Bt, cap)
            bf = self._buffers(Bt, W * cap, True)
            if c:
                bfc = self._buffers(c, W * cap, True)
                csr = self._csr(data, c, data.perm, self.boff)
                self._launch_pack_csr(bfc, csr, c / T)
            else:
                self._launch_pack_csr(None, None, 0.0)
            dp.communicate_csr()
            if c:
                self.accum_train.zero_()
                self._launch_fwd_bwd(bfc, csr, True, beta, p_drop, None)
                self._launch_pack_grads(bfc, c / T)
                sums = sums + self.accum_train.cpu().numpy() * (c / T)
            else:  # no users here: the union batch's plan still runs (and the schedule counter advances)
                self._resolve_pending()  # (no forward here to carry it; the apply below rewrites the rows it reads)
                dp.merge_plan()
                self._launch_pack_grads(None, 0.0)
                if anneal is not None:
                    ops.counter_add(self.anneal_dev, 1)
            dp.communicate_grads()
            self._launch_dp_update(bf, c)
            self.host_step += 1
        self.flush()
        dp.check()
        tot = dp.all_reduce(sums).tolist()  # the union batches' losses summed over the steps (Python floats:
        # the metrics go into checkpoints, which load with weights_only=True)
        return ({"total_loss": tot[0] / n_steps, "recon_loss": tot[1] / n_steps, "kl_loss": tot[2] / n_steps},
                n_steps)

    def _capture(self, bf: _StepBuffers, data: DeviceData, train: bool, beta: float, p_drop: float, key):
        """One graph per step (single GPU); data-parallel: the CSR packet | forward/backward (the union plan
        beside it) + the gradient packet | union apply + clip + Adam, with the collectives launched eagerly in
        between (they stay out of the graphs)."""
        csr = self._csr(data, bf.B, data.perm, self.boff)
        bf.csr_keepalive = csr
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        if self.dp is None or not train:
            with torch.cuda.graph(g):
                self._launch(bf, csr, train, beta, p_drop, advance=bf.B)
            bf.graph_pre = bf.graph_up = None
            k = self._steps_per_graph(bf.B) if self.dp is None else 1
            bf.graph_k, bf.graph_k_steps = None, 0
            if k > 1:  # the same step K times: each one reads the batch offset the previous one advanced
                gk = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gk):
                    for _ in range(k):
                        self._launch(bf, csr, train, beta, p_drop, advance=bf.B)
                bf.graph_k, bf.graph_k_steps = gk, k
        else:
            g0 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g0):
                self._launch_pack_csr(bf, csr, key[-1])
            with torch.cuda.graph(g):
                self._launch_fwd_bwd(bf, csr, train, beta, p_drop, None)
                self._launch_pack_grads(bf, key[-1])
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2):
                self._launch_dp_update(bf, bf.B)
            bf.graph_pre, bf.graph_up = g0, g2
        bf.graph = g
        bf.graph_key = key
        bf.graph_data = data

    def _steps_per_graph(self, B: int) -> int:
        """Steps per replay for batch size B: a step of a few hundred microseconds is host-bound on one replay
        per step (HVAE_STEPS_PER_GRAPH overrides)."""
        env = os.environ.get("HVAE_STEPS_PER_GRAPH")
        if env:
            return max(1, int(env))
        return 8 if B <= 1024 else 1

    def sync_state_to_model(self):
        """Parameters are views of the flat buffer already; nothing to copy."""
        return None


class ConstBeta:
    def __init__(self, beta: float):
        self.constant = float(beta)

    def __call__(self, _i):
        return self.constant


class AnnealedBeta:
    """AnnealedVAE's linear KL-weight schedule (reference src/ml/model.py:312-334) for a fused epoch.

    run_epoch evaluates it on the device (hvae_anneal_beta: one launch per train step that reads and advances a
    device copy of model.current_step), so annealed epochs replay one captured step like constant-beta ones, and
    then advances model.current_step by the steps it ran. Called directly (eager steps over other iterables) it is
    the reference's _compute_loss order: the current beta, then step_annealing()."""

    def __init__(self, model):
        self.model = model
        self.anneal = (float(model.beta_min), float(model.beta_max), int(model.anneal_steps))

    def __call__(self, _i):
        b = self.model.get_current_beta()
        self.model.step_annealing()
        return b
