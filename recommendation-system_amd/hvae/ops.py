"""Tensor-level wrappers of the libhvae C ABI.

Every function here takes/returns torch tensors that live on the HIP device,
checks shapes, allocates outputs, and launches on the current stream. They
are the building blocks of the module-API autograd path (hvae/autograd.py)
and of the parity tests. The fused trainer (hvae/executor.py) calls the C ABI
directly with preallocated buffers instead.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import (ROWSQ_PARTS, CsrBatch, Epilogue, RowGrad, Adam, check, lib, ptr, require_hip, stream_of)

_WS: dict[torch.device, torch.Tensor] = {}


def workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """Per-device scratch buffer, grown on demand (never shrunk)."""
    nbytes = max(int(nbytes), 256)
    ws = _WS.get(device)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(nbytes + (nbytes >> 2), dtype=torch.uint8, device=device)
        _WS[device] = ws
    return ws


class Csr:
    """A device CSR batch view (keeps the tensors alive for the C struct)."""

    def __init__(self, row_ptr: torch.Tensor, col_idx: torch.Tensor, vals: torch.Tensor, n_items: int,
                 rows: torch.Tensor | None = None, nb: int | None = None,
                 rows_offset: torch.Tensor | None = None):
        require_hip(row_ptr, col_idx, vals, rows)
        assert row_ptr.dtype == torch.int64 and col_idx.dtype == torch.int32 and vals.dtype == torch.float32
        assert rows is None or rows.dtype == torch.int32
        self.row_ptr, self.col_idx, self.vals, self.rows = row_ptr, col_idx, vals, rows
        self.rows_offset = rows_offset
        self.n_items = int(n_items)
        self.nb = int(nb if nb is not None else (rows.numel() if rows is not None else row_ptr.numel() - 1))
        self.struct = CsrBatch(ptr(row_ptr), ptr(col_idx), ptr(vals), ptr(rows), ptr(rows_offset), self.nb,
                               self.n_items)

    def rows_from_elsewhere(self):
        """The rows will be written by something other than the library's row-gradient apply (an injected
        DPExchange merge_fn): the clip must then read the rows, not the apply's per-row sums of squares
        (hvae_rowgrad.rowsq, include/hvae.h: non-NULL only where hvae_w1_rowgrad_apply produced the rows)."""
        self.struct.rowsq = None

    @property
    def ref(self):
        return C.byref(self.struct)


def csr_from_scipy(mat, device) -> Csr:
    """Upload a scipy.sparse CSR matrix (float values, summed duplicates kept) to the device."""
    mat = mat.tocsr()
    mat.sum_duplicates()
    row_ptr = torch.as_tensor(mat.indptr.astype("int64"), device=device)
    col = torch.as_tensor(mat.indices.astype("int32"), device=device)
    vals = torch.as_tensor(mat.data.astype("float32"), device=device)
    return Csr(row_ptr, col, vals, mat.shape[1])


def dense_to_csr(x: torch.Tensor) -> Csr:
    """Dense [B, N] (any values, zeros skipped) -> device CSR of the nonzeros."""
    require_hip(x)
    x = x.contiguous().float()
    B, N = x.shape
    cap = max(B * N, 1)
    row_ptr = torch.empty(B + 1, dtype=torch.int64, device=x.device)
    col = torch.empty(cap, dtype=torch.int32, device=x.device)
    vals = torch.empty(cap, dtype=torch.float32, device=x.device)
    check(lib().hvae_dense_to_csr(ptr(x), B, N, ptr(row_ptr), ptr(col), ptr(vals), cap, None, 0,
                                  stream_of(x)), "hvae_dense_to_csr")
    return Csr(row_ptr, col, vals, N)


# ------------------------------------------------------------------ encoder --
def encoder_fwd(x: Csr, w1t, b1, ln_w, ln_b, p_drop: float, train: bool, seed: int, step=None,
                drop_mult=None, save=True):
    H = w1t.shape[1]
    dev = w1t.device
    require_hip(w1t, b1, ln_w, ln_b, drop_mult)
    h = torch.empty(x.nb, H, device=dev)
    xhat = torch.empty(x.nb, H, device=dev) if save else None
    rstd = torch.empty(x.nb, device=dev) if save else None
    check(lib().hvae_encoder_fwd(x.ref, ptr(w1t), ptr(b1), ptr(ln_w), ptr(ln_b), H, float(p_drop), ptr(drop_mult),
                                 seed, ptr(step), int(train), ptr(h), ptr(xhat), ptr(rstd), stream_of(w1t)),
          "hvae_encoder_fwd")
    return h, xhat, rstd


def ln_gelu_drop_fwd(a, ln_w, ln_b, p_drop, train, seed, layer, step=None, drop_mult=None, save=True):
    require_hip(a, ln_w, ln_b, drop_mult)
    a = a.contiguous()
    nb, H = a.shape
    h = torch.empty_like(a)
    xhat = torch.empty_like(a) if save else None
    rstd = torch.empty(nb, device=a.device) if save else None
    check(lib().hvae_ln_gelu_drop_fwd(ptr(a), ptr(ln_w), ptr(ln_b), nb, H, float(p_drop), ptr(drop_mult), seed,
                                      ptr(step), layer, int(train), ptr(h), ptr(xhat), ptr(rstd), stream_of(a)),
          "hvae_ln_gelu_drop_fwd")
    return h, xhat, rstd


def ln_gelu_drop_bwd(dh, xhat, rstd, ln_w, ln_b, p_drop, train, seed, layer, step=None, drop_mult=None,
                     want_dbias=False):
    """-> (da, d_ln_w, d_ln_b) or, with want_dbias, (da, d_ln_w, d_ln_b, sum_rows(da))."""
    require_hip(dh, xhat, rstd, ln_w, ln_b)
    dh = dh.contiguous()
    nb, H = dh.shape
    da = torch.empty_like(dh)
    dw = torch.empty(H, device=dh.device)
    db = torch.empty(H, device=dh.device)
    dbias = torch.empty(H, device=dh.device) if want_dbias else None
    need = lib().hvae_ln_gelu_drop_bwd_workspace(nb, H)
    ws = workspace(dh.device, need)
    check(lib().hvae_ln_gelu_drop_bwd(ptr(dh), ptr(xhat), ptr(rstd), ptr(ln_w), ptr(ln_b), nb, H, float(p_drop),
                                      ptr(drop_mult), seed, ptr(step), layer, int(train), ptr(da), ptr(dw), ptr(db),
                                      ptr(dbias), ptr(ws), ws.numel(), stream_of(dh)), "hvae_ln_gelu_drop_bwd")
    return (da, dw, db, dbias) if want_dbias else (da, dw, db)


class RowGradBuffers:
    """Device buffers of the row-sparse first-layer weight gradient."""

    def __init__(self, n_items: int, H: int, cap: int, device, width: int | None = None):
        """width: the widest row the buffers must hold (default H): the fused step with trainable item embeddings
        also gathers rows of the decoder input u (width d) through the same plan."""
        W = max(H, width or H)
        i32 = dict(dtype=torch.int32, device=device)
        self.cnt = torch.zeros(n_items, **i32)
        self.slot_of = torch.full((n_items,), -1, **i32)
        self.item_of = torch.zeros(cap, **i32)
        self.seg_off = torch.zeros(cap + 1, **i32)
        self.fill = torch.zeros(cap, **i32)
        self.contrib_row = torch.zeros(cap, **i32)
        self.contrib_val = torch.zeros(cap, dtype=torch.float32, device=device)
        self.rows = torch.zeros(cap * W, dtype=torch.float32, device=device)[:cap * H].view(cap, H)
        self.n_unique = torch.zeros(1, **i32)
        self.contrib_slot = torch.zeros(cap, **i32)
        self.part = torch.empty(int(lib().hvae_rowgrad_part_floats(cap, W)), dtype=torch.float32, device=device)
        self.rowsq = torch.zeros(cap * ROWSQ_PARTS, dtype=torch.float64, device=device)
        self.cap, self.n_items, self.H = cap, n_items, H
        self.struct = RowGrad(ptr(self.cnt), ptr(self.slot_of), ptr(self.item_of), ptr(self.seg_off), ptr(self.fill),
                              ptr(self.contrib_row), ptr(self.contrib_val), ptr(self.rows), ptr(self.n_unique), cap,
                              n_items, ptr(self.contrib_slot), ptr(self.part), self.part.numel(), ptr(self.rowsq))
        self.ws = torch.empty(max(int(lib().hvae_w1_rowgrad_workspace(n_items)), 256), dtype=torch.uint8,
                              device=device)

    def rows_from_elsewhere(self):
        """The rows will be written by something other than the library's row-gradient apply (an injected
        DPExchange merge_fn): the clip must then read the rows, not the apply's per-row sums of squares
        (hvae_rowgrad.rowsq, include/hvae.h: non-NULL only where hvae_w1_rowgrad_apply produced the rows)."""
        self.struct.rowsq = None

    @property
    def ref(self):
        return C.byref(self.struct)


def w1_rowgrad(x: Csr, da: torch.Tensor, rg: RowGradBuffers) -> None:
    require_hip(da)
    check(lib().hvae_w1_rowgrad(x.ref, ptr(da), da.shape[1], rg.ref, ptr(rg.ws), rg.ws.numel(), stream_of(da)),
          "hvae_w1_rowgrad")


def w1_rowgrad_plan(x: Csr, rg: RowGradBuffers) -> None:
    """The plan half of w1_rowgrad (needs the batch only), on the current stream."""
    check(lib().hvae_w1_rowgrad_plan(x.ref, rg.ref, ptr(rg.ws), rg.ws.numel(),
                                     torch.cuda.current_stream(rg.rows.device).cuda_stream), "hvae_w1_rowgrad_plan")


def w1_rowgrad_apply(da: torch.Tensor, rg: RowGradBuffers) -> None:
    """The apply half of w1_rowgrad: rows from da over a plan already made."""
    require_hip(da)
    check(lib().hvae_w1_rowgrad_apply(ptr(da), da.shape[1], rg.ref, stream_of(da)), "hvae_w1_rowgrad_apply")


def rowgrad_to_dense(rg: RowGradBuffers, out: torch.Tensor) -> None:
    """out: zero-filled [N, ld] item-major buffer."""
    check(lib().hvae_rowgrad_to_dense(rg.ref, rg.H, ptr(out), out.stride(0), stream_of(out)),
          "hvae_rowgrad_to_dense")


# --------------------------------------------------------------------- GEMM --
def _as_operand(t: torch.Tensor):
    """(base tensor, transposed?, ld) such that t == base or t == base.T with base row-major."""
    if t.dim() != 2:
        raise ValueError("GEMM operands must be 2-D")
    if t.stride(1) == 1 and t.stride(0) >= max(t.shape[1], 1):
        return t, False, t.stride(0)
    if t.stride(0) == 1 and t.stride(1) >= max(t.shape[0], 1):
        return t, True, t.stride(1)
    return t.contiguous(), False, t.shape[1]


def gemm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, alpha=1.0, beta=0.0, epi=None):
    """out[M,N] = alpha * a[M,K] @ b[K,N] + beta * out (fp32 MFMA), then the epilogue.

    a and b may be transposed views (e.g. a Linear weight .t()); no copies are made.
    """
    require_hip(a, b)
    M, K = a.shape
    K2, N = b.shape
    assert K == K2, f"gemm shape mismatch {a.shape} @ {b.shape}"
    A, ta, lda = _as_operand(a)
    B, tb, ldb = _as_operand(b)
    if out is None:
        out = torch.empty(M, N, device=a.device)
        beta = 0.0
    assert out.stride(1) == 1
    need = lib().hvae_gemm_f32_workspace(M, N, K)
    ws = workspace(a.device, need) if need else None
    check(lib().hvae_gemm_f32(int(ta), int(tb), M, N, K, float(alpha), ptr(A), lda, ptr(B), ldb, float(beta),
                              ptr(out), out.stride(0), C.byref(epi) if epi is not None else None, ptr(ws),
                              ws.numel() if ws is not None else 0, stream_of(a)), "hvae_gemm_f32")
    return out


def epilogue(kind, bias=None, pre_out=None, pre_in=None, p_drop=0.0, drop_mult=None, seed=0, step=None,
             tag=0, train=False, opa_rowsum=None, aux=None, aux_scale=0.0, aux_scale_dev=None) -> Epilogue:
    return Epilogue(kind, ptr(bias), ptr(pre_out), ptr(pre_in), float(p_drop), ptr(drop_mult), int(seed), ptr(step),
                    int(tag), int(train), ptr(opa_rowsum), ptr(aux), float(aux_scale), ptr(aux_scale_dev))


def colsum(x: torch.Tensor, out: torch.Tensor | None = None, beta=0.0):
    require_hip(x)
    assert x.stride(1) == 1
    M, N = x.shape
    if out is None:
        out = torch.empty(N, device=x.device)
        beta = 0.0
    need = lib().hvae_colsum_workspace(M, N)
    ws = workspace(x.device, need)
    check(lib().hvae_colsum(ptr(x), M, N, x.stride(0), float(beta), ptr(out), ptr(ws), ws.numel(), stream_of(x)),
          "hvae_colsum")
    return out


# ------------------------------------------------------------------- latent --
def reparam_kl_fwd(mu, logvar, train: bool, seed: int, step=None, eps_in=None):
    require_hip(mu, logvar, eps_in)
    assert mu.stride(1) == 1 and logvar.stride(1) == 1 and mu.stride(0) == logvar.stride(0)
    nb, L = mu.shape
    z = torch.empty(nb, L, device=mu.device)
    eps = torch.empty(nb, L, device=mu.device) if train else None
    kl_rows = torch.empty(nb, device=mu.device)
    check(lib().hvae_reparam_kl_fwd(ptr(mu), ptr(logvar), mu.stride(0), nb, L, int(train), ptr(eps_in), seed,
                                    ptr(step), ptr(z), ptr(eps), ptr(kl_rows), stream_of(mu)), "hvae_reparam_kl_fwd")
    return z, eps, kl_rows


def reparam_kl_bwd(dz, mu, logvar, eps, kl_scale: float, train: bool, dmu=None, dlv=None, kl_scale_dev=None):
    nb, L = mu.shape
    if dmu is None:
        dmu = torch.empty(nb, L, device=mu.device)
        dlv = torch.empty(nb, L, device=mu.device)
    check(lib().hvae_reparam_kl_bwd(ptr(dz), ptr(mu), ptr(logvar), mu.stride(0), ptr(eps), nb, L, float(kl_scale),
                                    ptr(kl_scale_dev), int(train), ptr(dmu), ptr(dlv), dmu.stride(0), stream_of(mu)),
          "hvae_reparam_kl_bwd")
    return dmu, dlv


# ------------------------------------------------------------------ decoder --
class DecoderImage:
    """The frozen embeddings as the bf16 or fp8 decoder reads them (hvae_decoder_image): bf16 E [N, D]
    followed by its tile-transposed copy (bf16) or by the e4m3 fragment-order tiles and E's scale exponent
    (fp8). `bf16` is a view of the first part."""

    def __init__(self, E32: torch.Tensor, dtype: int = _lib.HVAE_BF16):
        require_hip(E32)
        if dtype not in (_lib.HVAE_BF16, _lib.HVAE_FP8):
            raise ValueError(f"decoder image dtype must be HVAE_BF16 or HVAE_FP8, got {dtype}")
        E32 = E32.contiguous()
        self.N, self.D = E32.shape
        self.dtype = dtype
        nbytes = int(lib().hvae_decoder_image_bytes(self.dtype, self.N, self.D))
        self.buf = torch.empty(nbytes, dtype=torch.uint8, device=E32.device)
        check(lib().hvae_decoder_image(self.dtype, ptr(E32), self.N, self.D, ptr(self.buf), stream_of(E32)),
              "hvae_decoder_image")
        self.bf16 = self.buf[: self.N * self.D * 2].view(torch.bfloat16).view(self.N, self.D)
        self.device = E32.device

    def refresh(self, E32: torch.Tensor) -> None:
        """Rewrite the image from new values of E in place (same shape; captured graphs keep their pointers)."""
        require_hip(E32)
        if tuple(E32.shape) != (self.N, self.D):
            raise ValueError(f"refresh: E shape {tuple(E32.shape)} != image shape {(self.N, self.D)}")
        E32 = E32.contiguous()
        check(lib().hvae_decoder_image(self.dtype, ptr(E32), self.N, self.D, ptr(self.buf), stream_of(E32)),
              "hvae_decoder_image")

    def data_ptr(self) -> int:
        return self.buf.data_ptr()


def decoder_image(E32: torch.Tensor, dtype: int = _lib.HVAE_BF16) -> DecoderImage:
    return DecoderImage(E32, dtype)


def _dec_operand(E):
    """(dtype code, N, pointer holder) of a decoder E argument: a DecoderImage (bf16) or an fp32 [N, D]."""
    if isinstance(E, DecoderImage):
        return E.dtype, E.N, E
    if E.dtype == torch.bfloat16:
        raise TypeError("the bf16 decoder takes a DecoderImage (ops.decoder_image), not a bf16 tensor")
    return _lib.HVAE_F32, E.shape[0], E


def row_norm_max(E, out: torch.Tensor | None = None) -> torch.Tensor:
    """max_i ||E_i|| of an fp32 / bf16 [N, D] matrix or of a DecoderImage's bf16 values (device scalar; written
    into `out` when given)."""
    if isinstance(E, DecoderImage):
        E = E.bf16
    require_hip(E)
    out = torch.empty(1, device=E.device) if out is None else out
    dtype = _lib.HVAE_BF16 if E.dtype == torch.bfloat16 else _lib.HVAE_F32
    check(lib().hvae_row_norm_max(dtype, ptr(E), E.shape[0], E.shape[1], ptr(out), stream_of(E)),
          "hvae_row_norm_max")
    return out


def cast_bf16(x: torch.Tensor) -> torch.Tensor:
    require_hip(x)
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    check(lib().hvae_cast_bf16(ptr(x), ptr(y), x.numel(), stream_of(x)), "hvae_cast_bf16")
    return y


def decoder_supported(dtype: int, D: int) -> bool:
    return bool(lib().hvae_decoder_supported(dtype, D))


def decoder_fwd(U: torch.Tensor, E, enorm: torch.Tensor | None, with_o: bool = True):
    """(lse [nb], O [nb, D] or None) of the streaming decoder; E a DecoderImage (bf16) or fp32 [N, D]."""
    dtype, N, Eh = _dec_operand(E)
    require_hip(U)
    assert U.stride(1) == 1
    nb, D = U.shape
    lse = torch.empty(nb, device=U.device)
    O = torch.empty(nb, D, device=U.device) if with_o else None
    need = lib().hvae_decoder_workspace(dtype, nb, N, D)
    ws = workspace(U.device, need)
    check(lib().hvae_decoder_fwd(dtype, ptr(U), U.stride(0), ptr(Eh), ptr(enorm), nb, N, D, ptr(lse), ptr(O),
                                 ptr(ws), ws.numel(), stream_of(U)), "hvae_decoder_fwd")
    return lse, O


def decoder_bwd(x: Csr, U, E32, lse, O, grad_scale: float, want_du: bool = True):
    nb, D = U.shape
    recon_rows = torch.empty(nb, device=U.device)
    dU = torch.empty(nb, D, device=U.device) if want_du else None
    check(lib().hvae_decoder_bwd(x.ref, ptr(U), U.stride(0), ptr(E32), D, ptr(lse), ptr(O), float(grad_scale),
                                 ptr(recon_rows), ptr(dU), stream_of(U)), "hvae_decoder_bwd")
    return recon_rows, dU


def decoder_train(x: Csr, U, E, enorm, E32, grad_scale: float, want_du: bool = True, want_o: bool = False,
                  kl_rows=None, beta: float = 0.0, loss3=None, accum3=None):
    """Fused sweep + finalize: (lse, O or None, recon_rows, dU or None).

    With kl_rows and loss3 given, the finalize also writes the batch loss means
    (total, recon, kl) into loss3 (and adds them to accum3), as hvae_loss_finalize.
    """
    dtype, N, Eh = _dec_operand(E)
    require_hip(U, E32)
    assert U.stride(1) == 1
    nb, D = U.shape
    lse = torch.empty(nb, device=U.device)
    O = torch.empty(nb, D, device=U.device) if want_o else None
    recon_rows = torch.empty(nb, device=U.device)
    dU = torch.empty(nb, D, device=U.device) if want_du else None
    ws = workspace(U.device, lib().hvae_decoder_workspace(dtype, nb, N, D))
    check(lib().hvae_decoder_train(dtype, ptr(U), U.stride(0), ptr(Eh), ptr(enorm), ptr(E32), x.ref, D,
                                   float(grad_scale), ptr(lse), ptr(O), ptr(recon_rows), ptr(dU), ptr(kl_rows),
                                   float(beta), None, ptr(loss3), ptr(accum3), ptr(ws), ws.numel(), stream_of(U)),
          "hvae_decoder_train")
    return lse, O, recon_rows, dU


def nll_rows_fwd(S, X):
    require_hip(S, X)
    nb, N = S.shape
    lse = torch.empty(nb, device=S.device)
    recon = torch.empty(nb, device=S.device)
    check(lib().hvae_nll_rows_fwd(ptr(S), S.stride(0), ptr(X), X.stride(0), nb, N, ptr(lse), ptr(recon),
                                  stream_of(S)), "hvae_nll_rows_fwd")
    return lse, recon


def nll_rows_bwd(S, X, lse, scale: float):
    nb, N = S.shape
    dS = torch.empty(nb, N, device=S.device)
    check(lib().hvae_nll_rows_bwd(ptr(S), S.stride(0), ptr(X), X.stride(0), ptr(lse), nb, N, float(scale), ptr(dS),
                                  dS.stride(0), stream_of(S)), "hvae_nll_rows_bwd")
    return dS


def loss_finalize(recon_rows, kl_rows, beta: float, out3=None, accum3=None):
    nb = recon_rows.numel()
    if out3 is None:
        out3 = torch.empty(3, device=recon_rows.device)
    check(lib().hvae_loss_finalize(ptr(recon_rows), ptr(kl_rows), nb, float(beta), ptr(out3), ptr(accum3),
                                   stream_of(recon_rows)), "hvae_loss_finalize")
    return out3


# ---------------------------------------------------------------- optimiser --
def clip_grad_norm(g_dense: torch.Tensor | None, rg: RowGradBuffers | None, max_norm: float,
                   norm_out=None, coef_out=None):
    dev = (g_dense if g_dense is not None else rg.rows).device
    if norm_out is None:
        norm_out = torch.empty(1, device=dev)
        coef_out = torch.empty(1, device=dev)
    n = g_dense.numel() if g_dense is not None else 0
    need = lib().hvae_clip_grad_norm_workspace(n, rg.cap if rg else 0, rg.H if rg else 0)
    ws = workspace(dev, need)
    check(lib().hvae_clip_grad_norm(ptr(g_dense), n, rg.ref if rg else None, rg.H if rg else 0, float(max_norm),
                                    ptr(norm_out), ptr(coef_out), ptr(ws), ws.numel(), torch.cuda.current_stream(
                                        dev).cuda_stream), "hvae_clip_grad_norm")
    return norm_out, coef_out


def adam_config(lr, betas, eps, weight_decay, step_dev, coef_dev=None) -> Adam:
    return Adam(float(lr), float(betas[0]), float(betas[1]), float(eps), float(weight_decay), ptr(step_dev),
                ptr(coef_dev))


def adam_dense(cfg: Adam, p, m, v, g):
    check(lib().hvae_adam_dense(C.byref(cfg), ptr(p), ptr(m), ptr(v), ptr(g), p.numel(), stream_of(p)),
          "hvae_adam_dense")


def adam_rows(cfg: Adam, p, m, v, rg: RowGradBuffers):
    N, H = p.shape
    check(lib().hvae_adam_rows(C.byref(cfg), ptr(p), ptr(m), ptr(v), rg.ref, N, H, stream_of(p)), "hvae_adam_rows")


def counter_add(c: torch.Tensor, delta: int = 1):
    check(lib().hvae_counter_add(ptr(c), int(delta), stream_of(c)), "hvae_counter_add")


# --------------------------------------------------------------------- eval --
def score_candidates(U, user_row, E32, cand):
    require_hip(U, user_row, E32, cand)
    R, Cn = cand.shape
    scores = torch.empty(R, Cn, device=U.device)
    check(lib().hvae_score_candidates(ptr(U), U.stride(0), ptr(user_row), ptr(E32), E32.shape[1], ptr(cand), R, Cn,
                                      ptr(scores), stream_of(U)), "hvae_score_candidates")
    return scores


def rank_first(scores):
    R, Cn = scores.shape
    rank = torch.empty(R, dtype=torch.int32, device=scores.device)
    check(lib().hvae_rank_first(ptr(scores), R, Cn, ptr(rank), stream_of(scores)), "hvae_rank_first")
    return rank


def topk(scores: torch.Tensor, k: int, exclude: Csr | None = None):
    """Exact top-k per row (score desc, ties -> larger index first); masks `exclude` in place."""
    require_hip(scores)
    R, N = scores.shape
    idx = torch.empty(R, k, dtype=torch.int32, device=scores.device)
    val = torch.empty(R, k, device=scores.device)
    check(lib().hvae_topk(ptr(scores), R, N, scores.stride(0), exclude.ref if exclude is not None else None, k,
                          ptr(idx), ptr(val), stream_of(scores)), "hvae_topk")
    return idx, val


def topk_fused(U: torch.Tensor, E_img: "DecoderImage", E32: torch.Tensor, e32_maxnorm: torch.Tensor, k: int,
               exclude: Csr | None = None, with_flags: bool = False):
    """Exact top-k of U E32^T per row (score desc, ties -> larger index first; `exclude`'s items of each row
    left out) without the [R, N] score matrix (hvae_topk_fused). Rows the fused path flags are ranked by the
    exact path (hvae_gemm_f32 scores + hvae_topk) for those rows only. Returns idx int32 [R, k], val [R, k]
    (and the flags when with_flags)."""
    require_hip(U, E32, e32_maxnorm)
    assert U.stride(1) == 1 and E32.is_contiguous()
    assert exclude is None or exclude.rows_offset is None
    R, D = U.shape
    N = E32.shape[0]
    idx = torch.empty(R, k, dtype=torch.int32, device=U.device)
    val = torch.empty(R, k, device=U.device)
    flag = torch.empty(R, dtype=torch.int32, device=U.device)
    ws = workspace(U.device, lib().hvae_topk_fused_workspace(R, N, D, k))
    check(lib().hvae_topk_fused(ptr(U), U.stride(0), ptr(E_img.bf16), ptr(E32), ptr(e32_maxnorm), N, D,
                                exclude.ref if exclude is not None else None, R, k, ptr(idx), ptr(val), ptr(flag),
                                ptr(ws), ws.numel(), stream_of(U)), "hvae_topk_fused")
    bad = torch.nonzero(flag).flatten()
    if bad.numel():
        rows = bad.to(torch.int32)
        S = gemm(U.index_select(0, bad), E32.t())
        ex = None
        if exclude is not None:
            sel = exclude.rows.index_select(0, bad) if exclude.rows is not None else rows
            ex = Csr(exclude.row_ptr, exclude.col_idx, exclude.vals, exclude.n_items, rows=sel.contiguous())
        i2, v2 = topk(S, k, exclude=ex)
        idx.index_copy_(0, bad, i2)
        val.index_copy_(0, bad, v2)
    return (idx, val, flag) if with_flags else (idx, val)


def negatives_legacy(indptr, indices, n_items: int, users, tests, n_neg: int, arrays: bool = False):
    """The 99-negative protocol's negatives for test rows (users[r], tests[r]) over a training CSR
    (indptr / indices), drawn by libhvae from numpy's global legacy RandomState exactly as the reference's
    per-row np.random.choice(available, n_neg, replace=False) would (src/ml/evaluate.py:159-170), which
    leaves the global state where those calls would have (hvae_negatives_legacy). Returns a list of int64
    arrays, one per row (shorter where fewer than n_neg items are available); with arrays=True the int32
    [rows, n_neg] block and the per-row counts instead (entries past a row's count are undefined)."""
    import numpy as np
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    users = np.ascontiguousarray(users, dtype=np.int32)
    tests = np.ascontiguousarray(tests, dtype=np.int32)
    R = len(users)
    st = np.random.get_state(legacy=True)
    if st[0] != "MT19937":
        raise RuntimeError(f"negatives_legacy: numpy global bit generator {st[0]}, not MT19937")
    key = np.array(st[1], dtype=np.uint32, copy=True)
    pos = np.array([st[2]], dtype=np.int32)
    out = np.empty((R, n_neg), dtype=np.int32)
    counts = np.empty(R, dtype=np.int32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    check(lib().hvae_negatives_legacy(p(key), p(pos), p(indptr), len(indptr) - 1, p(indices), int(n_items), p(users),
                                      p(tests), R, int(n_neg), p(out), p(counts)), "hvae_negatives_legacy")
    np.random.set_state((st[0], key, int(pos[0]), st[3], st[4]))
    if arrays:
        return out, counts
    return [out[r, :counts[r]].astype(np.int64) for r in range(R)]
