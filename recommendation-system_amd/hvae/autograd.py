"""torch.autograd.Functions over libhvae for the module API of HybridVAE.

This is the path of code that uses the model like the reference's own tests
do (model(x) -> scores, vae_loss_function(...), loss.backward()): every
forward and backward runs a libhvae kernel; only tensor bookkeeping is torch.
The training hot loop (VAETrainer) does not use these -- it runs the fused
graph-captured step of hvae/executor.py.

Reference: src/ml/model.py:138-256 (encode / reparameterize / decode /
forward / recommend) and :259-292 (vae_loss_function).
"""
from __future__ import annotations

import torch

from . import _lib, ops


def _seed() -> int:
    """Per-call Philox seed drawn from torch's default generator (torch.manual_seed reproducible)."""
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def _w1t(W1: torch.Tensor) -> torch.Tensor:
    """Item-major [N, H] image of encoder.0.weight [H, N] (free when stored item-major)."""
    w = W1.detach().t()
    return w if w.is_contiguous() else w.contiguous()


class EncoderFirstFn(torch.autograd.Function):
    """x (CSR) -> Dropout(GELU(LayerNorm(x W1^T + b1)))  (src/ml/model.py:112-118)."""

    @staticmethod
    def forward(ctx, W1, b1, ln_w, ln_b, csr: ops.Csr, p: float, train: bool):
        seed = _seed()
        h, xhat, rstd = ops.encoder_fwd(csr, _w1t(W1), b1.detach(), ln_w.detach(), ln_b.detach(), p, train, seed)
        ctx.save_for_backward(xhat, rstd, ln_w, ln_b)
        ctx.csr, ctx.p, ctx.train, ctx.seed, ctx.W1_shape = csr, p, train, seed, W1.shape
        return h

    @staticmethod
    def backward(ctx, dh):
        xhat, rstd, ln_w, ln_b = ctx.saved_tensors
        da, dlw, dlb, db1 = ops.ln_gelu_drop_bwd(dh, xhat, rstd, ln_w.detach(), ln_b.detach(), ctx.p, ctx.train,
                                                 ctx.seed, 0, want_dbias=True)
        dW1 = None
        if ctx.needs_input_grad[0]:
            H, N = ctx.W1_shape
            rg = ops.RowGradBuffers(N, H, max(int(ctx.csr.row_ptr[-1].item()), 1), da.device)
            ops.w1_rowgrad(ctx.csr, da, rg)
            dense = torch.zeros(N, H, device=da.device)
            ops.rowgrad_to_dense(rg, dense)
            dW1 = dense.t()
        return dW1, db1, dlw, dlb, None, None, None


class LinearFn(torch.autograd.Function):
    """y = x W^T + b, optionally fused with GELU + Dropout (nn.Linear [+ GELU + Dropout])."""

    @staticmethod
    def forward(ctx, x, W, b, act: bool, p: float, train: bool):
        x = x.contiguous()
        ctx.act, ctx.p, ctx.train = act, p, train
        if act:
            seed = _seed()
            pre = torch.empty(x.shape[0], W.shape[0], device=x.device)
            epi = ops.epilogue(_lib.EPI_BIAS_GELU_DROP, bias=b.detach(), pre_out=pre, p_drop=p, seed=seed,
                               tag=_lib.TAG_PROJ_DROP, train=train)
            y = ops.gemm(x, W.detach().t(), epi=epi)
            ctx.seed = seed
            ctx.save_for_backward(x, W, pre)
        else:
            epi = ops.epilogue(_lib.EPI_BIAS, bias=b.detach())
            y = ops.gemm(x, W.detach().t(), epi=epi)
            ctx.save_for_backward(x, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        if ctx.act:
            x, W, pre = ctx.saved_tensors
            # d(pre) = dy * dropout * GELU'(pre): the GEMM epilogue applies it while copying dy through an
            # identity product (module-API path only; the fused trainer folds it into the dq GEMM)
            eye_epi = ops.epilogue(_lib.EPI_GELU_DROP_BWD, pre_in=pre, p_drop=ctx.p, seed=ctx.seed,
                                   tag=_lib.TAG_PROJ_DROP, train=ctx.train)
            eye = torch.eye(dy.shape[1], device=dy.device)
            dpre = ops.gemm(dy, eye, epi=eye_epi)
        else:
            x, W = ctx.saved_tensors
            dpre = dy
        dx = ops.gemm(dpre, W.detach()) if ctx.needs_input_grad[0] else None
        db = torch.empty(W.shape[0], device=dy.device) if ctx.needs_input_grad[2] else None
        dW = ops.gemm(dpre.t(), x, epi=ops.epilogue(_lib.EPI_NONE, opa_rowsum=db))  # bias grad rides along
        if not ctx.needs_input_grad[1]:
            dW = None
        return dx, dW, db, None, None, None


class LnGeluDropFn(torch.autograd.Function):
    """Dropout(GELU(LayerNorm(a))) for hidden layers >= 2 (src/ml/model.py:115-117)."""

    @staticmethod
    def forward(ctx, a, ln_w, ln_b, p: float, train: bool, layer: int):
        seed = _seed()
        h, xhat, rstd = ops.ln_gelu_drop_fwd(a, ln_w.detach(), ln_b.detach(), p, train, seed, layer)
        ctx.save_for_backward(xhat, rstd, ln_w, ln_b)
        ctx.p, ctx.train, ctx.seed, ctx.layer = p, train, seed, layer
        return h

    @staticmethod
    def backward(ctx, dh):
        xhat, rstd, ln_w, ln_b = ctx.saved_tensors
        da, dlw, dlb = ops.ln_gelu_drop_bwd(dh, xhat, rstd, ln_w.detach(), ln_b.detach(), ctx.p, ctx.train, ctx.seed,
                                            ctx.layer)
        return da, dlw, dlb, None, None, None


class ReparamFn(torch.autograd.Function):
    """z = mu + eps * exp(0.5 logvar), eps ~ N(0, 1)  (src/ml/model.py:168-176)."""

    @staticmethod
    def forward(ctx, mu, logvar):
        mu, logvar = mu.contiguous(), logvar.contiguous()
        z, eps, _ = ops.reparam_kl_fwd(mu, logvar, True, _seed())
        ctx.save_for_backward(mu, logvar, eps)
        return z

    @staticmethod
    def backward(ctx, dz):
        mu, logvar, eps = ctx.saved_tensors
        dmu, dlv = ops.reparam_kl_bwd(dz.contiguous(), mu, logvar, eps, 0.0, True)
        return dmu, dlv


class ScoresFn(torch.autograd.Function):
    """scores = u E^T  (src/ml/model.py:198); dE only if E is trainable."""

    @staticmethod
    def forward(ctx, u, E):
        u = u.contiguous()
        ctx.save_for_backward(u, E)
        return ops.gemm(u, E.detach().t())

    @staticmethod
    def backward(ctx, dS):
        u, E = ctx.saved_tensors
        dS = dS.contiguous()
        du = ops.gemm(dS, E.detach()) if ctx.needs_input_grad[0] else None
        dE = ops.gemm(dS.t(), u) if ctx.needs_input_grad[1] else None
        return du, dE


class VaeLossFn(torch.autograd.Function):
    """(total, recon, kl) of vae_loss_function (src/ml/model.py:259-292) on materialised scores."""

    @staticmethod
    def forward(ctx, S, x, mu, logvar, beta: float):
        S, x = S.contiguous(), x.contiguous().float()
        mu, logvar = mu.contiguous(), logvar.contiguous()
        lse, recon_rows = ops.nll_rows_fwd(S, x)
        _, _, kl_rows = ops.reparam_kl_fwd(mu, logvar, False, 0)
        out3 = ops.loss_finalize(recon_rows, kl_rows, beta)
        ctx.save_for_backward(S, x, lse, mu, logvar)
        ctx.beta = beta
        return out3[0], out3[1], out3[2]

    @staticmethod
    def backward(ctx, g_total, g_recon, g_kl):
        S, x, lse, mu, logvar = ctx.saved_tensors
        B = S.shape[0]
        gt = 0.0 if g_total is None else float(g_total)
        gr = 0.0 if g_recon is None else float(g_recon)
        gk = 0.0 if g_kl is None else float(g_kl)
        dS = ops.nll_rows_bwd(S, x, lse, (gt + gr) / B) if ctx.needs_input_grad[0] else None
        dmu = dlv = None
        if ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            dmu, dlv = ops.reparam_kl_bwd(None, mu, logvar, None, (ctx.beta * gt + gk) / B, False)
        return dS, None, dmu, dlv, None
