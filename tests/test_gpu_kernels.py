"""Per-kernel parity of libhvae (through the C ABI) against CPU fp32 references.

Each HIP op is compared with a plain fp32 PyTorch-on-CPU statement of the same
op (the oracle's building blocks). Integer/index work is checked bit-exact.
"""
import ctypes as C
import math

import numpy as np
import pytest
import torch

from gen import synth_csr, synth_embeddings
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(hip_device):
    from hvae import ops
    return ops


def _maxrel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-30))


# ------------------------------------------------------------------ GEMM ---
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (7, 13, 5), (64, 64, 64), (130, 67, 300), (37, 384, 4096),
                                   (384, 384, 4096), (4096, 128, 512),
                                   # weight-gradient fast path (trans_a, K >= 1024): 32- and 64-square tiles
                                   (768, 768, 4096), (256, 64, 2048),
                                   # whole 64-tiles (the LDS-DMA path's 64 x 64 instance)
                                   (4096, 768, 256),
                                   # the LDS-DMA path's 64 x 32 tile (no trans_a, 256 64-square tiles, 512 64 x 32
                                   # ones: the Syn-10M step's heads / dh shapes)
                                   (4096, 256, 512)])
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm_f32(ops, hip_device, M, N, K, ta, tb):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    Ad = (A.t().contiguous().to(hip_device).t() if ta else A.to(hip_device))
    Bd = (B.t().contiguous().to(hip_device).t() if tb else B.to(hip_device))
    C0 = torch.randn(M, N, generator=g)
    out = C0.to(hip_device).clone()
    ops.gemm(Ad, Bd, out=out, alpha=0.5, beta=0.25)
    ref = 0.5 * (A.double() @ B.double()) + 0.25 * C0.double()
    assert _maxrel(out, ref) < 2e-5 * max(1.0, math.sqrt(K) / 8)


@pytest.mark.parametrize("M,N,K", [(50, 70, 33), (128, 96, 64), (4096, 256, 512)])
def test_gemm_epilogues(ops, hip_device, M, N, K):
    """The fused epilogues on a ragged shape (register-staged kernel) and whole-tile ones (LDS-DMA path: 32 x 32
    at 128 x 96, the 64 x 32 tile at 4096 x 256; split-K is never planned without trans_a)."""
    from hvae import _lib
    g = torch.Generator().manual_seed(3)
    A, W, bias = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g), torch.randn(N, generator=g)
    mult = ((torch.rand(M, N, generator=g) >= 0.3).float() / 0.7)
    Ad, Wd, bd, md = (t.to(hip_device) for t in (A, W, bias, mult))
    pre = torch.empty(M, N, device=hip_device)
    epi = ops.epilogue(_lib.EPI_BIAS_GELU_DROP, bias=bd, pre_out=pre, p_drop=0.3, drop_mult=md, train=True)
    out = ops.gemm(Ad, Wd.t(), epi=epi)
    ref_pre = A @ W.t() + bias
    assert _maxrel(pre, ref_pre) < 1e-5
    assert _maxrel(out, R.gelu(ref_pre) * mult) < 1e-5
    # backward epilogue: c * mult * gelu'(pre)
    G, W2 = torch.randn(M, 64, generator=g), torch.randn(64, N, generator=g)
    epi2 = ops.epilogue(_lib.EPI_GELU_DROP_BWD, pre_in=pre, p_drop=0.3, drop_mult=md, train=True)
    out2 = ops.gemm(G.to(hip_device), W2.to(hip_device), epi=epi2)
    x = ref_pre.clone().requires_grad_(True)
    (R.gelu(x) * mult * (G @ W2)).sum().backward()
    assert _maxrel(out2, x.grad) < 1e-5


@pytest.mark.parametrize("M,N,K", [(384, 384, 64), (256, 512, 4096), (70, 33, 5)])
def test_gemm_tn_bias_rowsum(ops, hip_device, M, N, K):
    """dW = dY^T X with the bias gradient sum_k dY[k, m] computed from the same staged tiles."""
    from hvae import _lib
    g = torch.Generator().manual_seed(M + K)
    dY, X = torch.randn(K, M, generator=g), torch.randn(K, N, generator=g)
    rs = torch.empty(M, device=hip_device)
    out = ops.gemm(dY.to(hip_device).t(), X.to(hip_device), epi=ops.epilogue(_lib.EPI_NONE, opa_rowsum=rs))
    assert _maxrel(out, dY.double().t() @ X.double()) < 2e-5 * max(1.0, math.sqrt(K) / 8)
    assert _maxrel(rs, dY.double().sum(0)) < 1e-5


@pytest.mark.parametrize("B,M,N,Kx", [(64, 384, 384, 384), (4096, 256, 512, 256), (64, 384, 128, 384),
                                     (50, 70, 33, 45), (4096, 768, 768, 768), (2048, 768, 128, 768)])
def test_gemm_pair_equals_two_launches(ops, hip_device, B, M, N, Kx):
    """hvae_gemm_f32_pair (dW = dY^T X with the bias gradient, and dX = dY W in one launch) is bitwise the
    two hvae_gemm_f32 launches it replaces, including split-K on the weight gradient at large B."""
    import ctypes as C
    from hvae import _lib
    from hvae._lib import GemmDesc, check, lib, ptr, stream_of
    g = torch.Generator().manual_seed(B + M)
    dY = torch.randn(B, M, generator=g).to(hip_device)
    X = torch.randn(B, N, generator=g).to(hip_device)
    W = torch.randn(M, Kx, generator=g).to(hip_device)
    rs1 = torch.empty(M, device=hip_device)
    dW1 = ops.gemm(dY.t(), X, epi=ops.epilogue(_lib.EPI_NONE, opa_rowsum=rs1))
    dX1 = ops.gemm(dY, W)
    rs2 = torch.empty(M, device=hip_device)
    dW2 = torch.empty(M, N, device=hip_device)
    dX2 = torch.empty(B, Kx, device=hip_device)
    ws = ops.workspace(hip_device, int(lib().hvae_gemm_f32_workspace(M, N, B)))
    epi = _lib.Epilogue(_lib.EPI_NONE, None, None, None, 0.0, None, 0, None, 0, 0, ptr(rs2))
    dw = GemmDesc(1, 0, M, N, B, 1.0, ptr(dY), M, ptr(X), N, 0.0, ptr(dW2), N, C.pointer(epi), ptr(ws), ws.numel())
    dx = GemmDesc(0, 0, B, Kx, M, 1.0, ptr(dY), M, ptr(W), Kx, 0.0, ptr(dX2), Kx, None, None, 0)
    check(lib().hvae_gemm_f32_pair(C.byref(dw), C.byref(dx), stream_of(dY)), "gemm_pair")
    torch.cuda.synchronize()
    assert torch.equal(dW1, dW2) and torch.equal(rs1, rs2) and torch.equal(dX1, dX2)


def test_colsum(ops, hip_device):
    X = torch.randn(3000, 77)
    out = ops.colsum(X.to(hip_device))
    assert _maxrel(out, X.double().sum(0)) < 1e-5


# --------------------------------------------------------------- encoder ---
def _csr_dev(ops, X, device):
    return ops.csr_from_scipy(X, device)


@pytest.mark.parametrize("H", [64, 128, 512, 600])
def test_encoder_fwd_bwd(ops, hip_device, H):
    X = synth_csr(37, 500, lam=6.0, seed=1)
    x = torch.as_tensor(X.toarray(), dtype=torch.float32)
    g = torch.Generator().manual_seed(H)
    W1 = torch.randn(H, 500, generator=g) * 0.05
    b1, lw, lb = torch.randn(H, generator=g), 1 + 0.1 * torch.randn(H, generator=g), torch.randn(H, generator=g)
    mult = ((torch.rand(37, H, generator=g) >= 0.25).float() / 0.75)
    xd = _csr_dev(ops, X, hip_device)
    w1t = W1.t().contiguous().to(hip_device)
    dv = lambda t: t.to(hip_device)
    h, xhat, rstd = ops.encoder_fwd(xd, w1t, dv(b1), dv(lw), dv(lb), 0.25, True, 0, drop_mult=dv(mult))
    a = (x @ W1.t() + b1).requires_grad_(True)
    ref = R.gelu(R.layer_norm(a, lw, lb)) * mult
    assert _maxrel(h, ref) < 2e-5
    # backward through LN/GELU/dropout + row-sparse W1 grad
    dh = torch.randn(37, H, generator=g)
    lw_ = lw.clone().requires_grad_(True)
    lb_ = lb.clone().requires_grad_(True)
    (R.gelu(R.layer_norm(a, lw_, lb_)) * mult * dh).sum().backward()
    da, dlw, dlb, dbias = ops.ln_gelu_drop_bwd(dv(dh), xhat, rstd, dv(lw), dv(lb), 0.25, True, 0, 0,
                                               drop_mult=dv(mult), want_dbias=True)
    assert _maxrel(da, a.grad) < 5e-5
    assert _maxrel(dbias, a.grad.sum(0)) < 5e-5
    assert _maxrel(dlw, lw_.grad) < 5e-5 and _maxrel(dlb, lb_.grad) < 5e-5
    rg = ops.RowGradBuffers(500, H, int(X.nnz), hip_device)
    ops.w1_rowgrad(xd, da, rg)
    dense = torch.zeros(500, H, device=hip_device)
    ops.rowgrad_to_dense(rg, dense)
    ref_w1 = (a.grad.t() @ x).t()  # [N, H]
    assert _maxrel(dense, ref_w1) < 5e-5
    # slots are the touched items in ascending order, bit-exact
    nu = int(rg.n_unique.item())
    touched = np.unique(X.indices)
    assert nu == len(touched)
    np.testing.assert_array_equal(rg.item_of[:nu].cpu().numpy(), touched)
    assert int(rg.cnt.abs().sum()) == 0 and int(rg.fill.abs().sum()) == 0
    # determinism: a second run is bitwise identical
    rows1 = rg.rows[:nu].clone()
    ops.w1_rowgrad(xd, da, rg)
    assert torch.equal(rows1, rg.rows[:nu])


def test_philox_dropout_statistics(ops, hip_device):
    X = synth_csr(256, 300, seed=2)
    xd = _csr_dev(ops, X, hip_device)
    H = 512
    w1t = torch.randn(300, H, device=hip_device) * 0.05
    one, zero = torch.ones(H, device=hip_device), torch.zeros(H, device=hip_device)
    step = torch.zeros(1, dtype=torch.int64, device=hip_device)
    h0, _, _ = ops.encoder_fwd(xd, w1t, zero, one, zero, 0.0, True, 7, step=step)
    h1, _, _ = ops.encoder_fwd(xd, w1t, zero, one, zero, 0.3, True, 7, step=step)
    keep = (h1 != 0) | (h0 == 0)
    frac = keep.float().mean().item()
    assert abs(frac - 0.7) < 0.01
    kept = h1[(h1 != 0)]
    assert torch.allclose(kept, h0[(h1 != 0)] / 0.7, rtol=1e-5, atol=1e-6)
    # same (seed, step) -> same mask; next step -> a different one
    h2, _, _ = ops.encoder_fwd(xd, w1t, zero, one, zero, 0.3, True, 7, step=step)
    assert torch.equal(h1, h2)
    step += 1
    h3, _, _ = ops.encoder_fwd(xd, w1t, zero, one, zero, 0.3, True, 7, step=step)
    assert not torch.equal(h1, h3)


def test_dense_to_csr(ops, hip_device):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(9, 1000, generator=g) * (torch.rand(9, 1000, generator=g) < 0.05)
    x[3] = 0
    c = ops.dense_to_csr(x.to(hip_device))
    rp = c.row_ptr.cpu().numpy()
    nz = [np.nonzero(r)[0] for r in x.numpy()]
    np.testing.assert_array_equal(np.diff(rp), [len(z) for z in nz])
    np.testing.assert_array_equal(c.col_idx[: rp[-1]].cpu().numpy(), np.concatenate(nz))
    np.testing.assert_array_equal(c.vals[: rp[-1]].cpu().numpy(), x.numpy()[x.numpy() != 0])


# ---------------------------------------------------------------- latent ---
def test_reparam_kl(ops, hip_device):
    g = torch.Generator().manual_seed(5)
    B, L = 33, 64
    heads = torch.randn(B, 2 * L, generator=g)
    eps = torch.randn(B, L, generator=g)
    hd = heads.to(hip_device)
    mu, lv = hd[:, :L], hd[:, L:]
    z, eps_o, kl_rows = ops.reparam_kl_fwd(mu, lv, True, 0, eps_in=eps.to(hip_device))
    m_, l_ = heads[:, :L].clone().requires_grad_(True), heads[:, L:].clone().requires_grad_(True)
    zr = m_ + eps * torch.exp(0.5 * l_)
    klr = -0.5 * (1 + l_ - m_ ** 2 - l_.exp()).sum(1)
    assert _maxrel(z, zr) < 1e-6 and _maxrel(kl_rows, klr) < 1e-5
    dz = torch.randn(B, L, generator=g)
    beta = 0.2
    (zr * dz).sum().add(beta * klr.sum() / B).backward()
    dmu, dlv = ops.reparam_kl_bwd(dz.to(hip_device), mu, lv, eps_o, beta / B, True)
    assert _maxrel(dmu, m_.grad) < 1e-5 and _maxrel(dlv, l_.grad) < 1e-5
    # the same backward as the epilogue of the GEMM that produces dz (dz = G W): [dmu | dlogvar]
    from hvae import _lib
    Gm, W = torch.randn(B, 96, generator=g), torch.randn(96, L, generator=g)
    dz2 = (Gm @ W).to(hip_device)
    dmu2, dlv2 = ops.reparam_kl_bwd(dz2, mu, lv, eps_o, beta / B, True)
    dheads = torch.empty(B, 2 * L, device=hip_device)
    epi = ops.epilogue(_lib.EPI_REPARAM_BWD, pre_in=hd, train=True, aux=eps_o, aux_scale=beta / B)
    ops.gemm(Gm.to(hip_device), W.to(hip_device), out=dheads, epi=epi)
    assert _maxrel(dheads[:, :L], dmu2) < 1e-5 and _maxrel(dheads[:, L:], dlv2) < 1e-5


# --------------------------------------------------------------- decoder ---
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("nb,N,D", [(3, 50, 384), (64, 890, 384), (200, 12101, 384), (130, 1000, 128),
                                    (17, 333, 64), (300, 5000, 256), (129, 777, 384), (300, 5001, 384)])
def test_decoder(ops, hip_device, dtype, nb, N, D):
    """Every sweep against float64 (bf16: on the bf16-rounded operands): partial last user blocks, item tails,
    1 .. 8 splits."""
    _check_decoder(ops, hip_device, dtype, nb, N, D)


@pytest.mark.parametrize("nb,N,D", [(64, 2000, 768), (300, 5001, 768), (7, 100, 768)])
def test_decoder_bf16_d768(ops, hip_device, nb, N, D):
    """Syn-10M's d = 768 (BASELINE configs[3]): the D-split bf16 sweep (two waves per user group)."""
    _check_decoder(ops, hip_device, "bf16", nb, N, D)


def _check_decoder(ops, hip_device, dtype, nb, N, D):
    E = torch.as_tensor(synth_embeddings(N, D, seed=N))
    g = torch.Generator().manual_seed(nb)
    U = torch.randn(nb, D, generator=g) * 3.0
    Ed = E.to(hip_device)
    Ek = ops.decoder_image(Ed) if dtype == "bf16" else Ed
    if dtype == "bf16":
        Ur, Er = U.bfloat16().float(), Ek.bf16.float().cpu()
    else:
        Ur, Er = U, E
    enorm = ops.row_norm_max(Ek)
    lse, O = ops.decoder_fwd(U.to(hip_device), Ek, enorm)
    S = Ur.double() @ Er.double().t()
    lse_ref = torch.logsumexp(S, 1)
    O_ref = torch.softmax(S, 1) @ Er.double()
    tol = 1e-5 if dtype == "f32" else 2e-3
    assert (lse.double().cpu() - lse_ref).abs().max() < tol * max(1.0, lse_ref.abs().max().item())
    assert _maxrel(O, O_ref) < (1e-5 if dtype == "f32" else 1e-2)
    lse2, _ = ops.decoder_fwd(U.to(hip_device), Ek, enorm, with_o=False)
    assert torch.allclose(lse2, lse, rtol=0, atol=1e-5)


@pytest.mark.parametrize("D,reps", [(128, 1), (384, 12)])
def test_decoder_large_norm_fixup(ops, hip_device, D, reps):
    """|u| in the hundreds: the fixed-offset bf16 path must flag and fix underflowing users (d = 384 with 96
    users: the DS = 1 sweep's flags)."""
    N = 4000
    E = torch.as_tensor(synth_embeddings(N, D, seed=9))
    g = torch.Generator().manual_seed(1)
    U = torch.randn(8 * reps, D, generator=g)
    U = U / U.norm(dim=1, keepdim=True) * torch.tensor([1, 10, 50, 100, 200, 400, 800, 1500.0]).repeat(reps)[:, None]
    Ek = ops.decoder_image(E.to(hip_device))
    lse, O = ops.decoder_fwd(U.to(hip_device), Ek, ops.row_norm_max(Ek))
    S = U.bfloat16().double() @ Ek.bf16.float().cpu().double().t()
    assert torch.isfinite(lse).all() and torch.isfinite(O).all()
    rel = ((lse.double().cpu() - torch.logsumexp(S, 1)).abs() / torch.logsumexp(S, 1).abs().clamp(min=1))
    assert rel.max() < 2e-3
    # the fused train form recomputes flagged users inside its finalize: same lse, O-derived dU
    X = synth_csr(8 * reps, N, lam=5.0, seed=2)
    xd = ops.csr_from_scipy(X, hip_device)
    Ed = E.to(hip_device)
    sc = 1.0 / (8 * reps)
    lse_t, O_t, _, dU_t = ops.decoder_train(xd, U.to(hip_device), Ek, ops.row_norm_max(Ek), Ed, sc, want_o=True)
    assert torch.equal(lse_t, lse) and torch.equal(O_t, O)
    _, _, _, dU_n = ops.decoder_train(xd, U.to(hip_device), Ek, ops.row_norm_max(Ek), Ed, sc)
    assert torch.equal(dU_n, dU_t)


def test_decoder_bwd_sparse(ops, hip_device):
    X = synth_csr(40, 700, lam=5.0, seed=4)
    x = torch.as_tensor(X.toarray(), dtype=torch.float32)
    D = 384
    E = torch.as_tensor(synth_embeddings(700, D, seed=3))
    U = torch.randn(40, D) * 2
    xd = ops.csr_from_scipy(X, hip_device)
    Ed = E.to(hip_device)
    lse, O = ops.decoder_fwd(U.to(hip_device), Ed, None)
    recon_rows, dU = ops.decoder_bwd(xd, U.to(hip_device), Ed, lse, O, 1.0 / 40)
    u_ = U.clone().requires_grad_(True)
    S = u_ @ E.t()
    rr = -(x * torch.log_softmax(S, 1)).sum(1)
    rr.mean().backward()
    assert _maxrel(recon_rows, rr) < 1e-5
    assert _maxrel(dU, u_.grad) < 1e-4


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("nb,N,D", [(40, 700, 384), (64, 12101, 384), (5, 3000, 128), (256, 2000, 64),
                                    (130, 4001, 384)])
def test_decoder_train_fused(ops, hip_device, dtype, nb, N, D):
    _check_decoder_train_fused(ops, hip_device, dtype, nb, N, D)


@pytest.mark.parametrize("nb,N,D", [(64, 3000, 768), (130, 4000, 768)])
def test_decoder_train_fused_d768(ops, hip_device, nb, N, D):
    _check_decoder_train_fused(ops, hip_device, "bf16", nb, N, D)


def _check_decoder_train_fused(ops, hip_device, dtype, nb, N, D):
    """Sweep + merge + sparse terms in one finalize launch == decoder_fwd + decoder_bwd == torch autograd."""
    X = synth_csr(nb, N, lam=5.0, seed=nb + N)
    x = torch.as_tensor(X.toarray(), dtype=torch.float32)
    E = torch.as_tensor(synth_embeddings(N, D, seed=3))
    g = torch.Generator().manual_seed(5)
    U = torch.randn(nb, D, generator=g) * 2
    xd = ops.csr_from_scipy(X, hip_device)
    Ed, Ud = E.to(hip_device), U.to(hip_device)
    Ek = ops.decoder_image(Ed) if dtype == "bf16" else Ed
    enorm = ops.row_norm_max(Ek)
    lse, O, rr, dU = ops.decoder_train(xd, Ud, Ek, enorm, Ed, 1.0 / nb, want_o=True)
    lse_b, O_b = ops.decoder_fwd(Ud, Ek, enorm)
    rr_b, dU_b = ops.decoder_bwd(xd, Ud, Ed, lse_b, O_b, 1.0 / nb)
    assert torch.equal(lse, lse_b) and torch.equal(rr, rr_b) and torch.equal(dU, dU_b) and torch.equal(O, O_b)
    _, _, rr2, dU2 = ops.decoder_train(xd, Ud, Ek, enorm, Ed, 1.0 / nb)  # O kept internal
    assert torch.equal(rr2, rr) and torch.equal(dU2, dU)
    _, _, rr3, none = ops.decoder_train(xd, Ud, Ek, enorm, Ed, 1.0 / nb, want_du=False)
    assert none is None and torch.equal(rr3, rr)
    # the batch loss means fused into the finalize == hvae_loss_finalize on the same rows
    kl = torch.rand(nb, generator=g).to(hip_device)
    loss3 = torch.empty(3, device=hip_device)
    acc3 = torch.zeros(3, dtype=torch.float64, device=hip_device)
    _, _, rr4, dU4 = ops.decoder_train(xd, Ud, Ek, enorm, Ed, 1.0 / nb, kl_rows=kl, beta=0.2, loss3=loss3,
                                       accum3=acc3)
    assert torch.equal(rr4, rr) and torch.equal(dU4, dU)
    ref3 = ops.loss_finalize(rr, kl, 0.2)
    assert torch.equal(loss3, ref3) and torch.equal(acc3.float(), ref3)
    u_ = U.clone().requires_grad_(True)
    rr_t = -(x * torch.log_softmax(u_ @ E.t(), 1)).sum(1)
    rr_t.mean().backward()
    tol = (1e-5, 1e-4) if dtype == "f32" else (3e-3, 2e-2)
    assert _maxrel(rr, rr_t) < tol[0]
    assert _maxrel(dU, u_.grad) < tol[1]


def test_nll_rows(ops, hip_device):
    g = torch.Generator().manual_seed(2)
    S = torch.randn(6, 77, generator=g) * 3
    X = torch.randn(6, 77, generator=g)  # reference tests feed randn inputs
    lse, rr = ops.nll_rows_fwd(S.to(hip_device), X.to(hip_device))
    s_ = S.clone().requires_grad_(True)
    ref = -(X * torch.log_softmax(s_, 1)).sum(1)
    ref.mean().backward()
    assert _maxrel(rr, ref) < 1e-5
    dS = ops.nll_rows_bwd(S.to(hip_device), X.to(hip_device), lse, 1.0 / 6)
    assert _maxrel(dS, s_.grad) < 1e-5


# ------------------------------------------------------------- optimiser ---
def test_clip_and_adam(ops, hip_device):
    g = torch.Generator().manual_seed(4)
    N, H = 300, 64
    small = torch.randn(5000, generator=g)
    X = synth_csr(20, N, seed=5)
    xd = ops.csr_from_scipy(X, hip_device)
    da = torch.randn(20, H, generator=g)
    rg = ops.RowGradBuffers(N, H, int(X.nnz), hip_device)
    ops.w1_rowgrad(xd, da.to(hip_device), rg)
    dense = torch.zeros(N, H, device=hip_device)
    ops.rowgrad_to_dense(rg, dense)
    w1g = dense.cpu()
    total_ref = math.sqrt(float((small.double() ** 2).sum() + (w1g.double() ** 2).sum()))
    norm, coef = ops.clip_grad_norm(small.to(hip_device), rg, 5.0)
    assert abs(norm.item() - total_ref) < 1e-5 * total_ref
    assert abs(coef.item() - min(1.0, 5.0 / (total_ref + 1e-6))) < 1e-6
    # Adam: dense segment and row-sparse W1t, 3 steps, vs the oracle's torch.optim.Adam restatement
    step = torch.zeros(1, dtype=torch.int64, device=hip_device)
    cfg = ops.adam_config(1e-3, (0.9, 0.999), 1e-8, 0.0, step, coef)
    p_s, p_w = torch.randn(5000, generator=g), torch.randn(N, H, generator=g)
    ps_d, pw_d = p_s.to(hip_device), p_w.to(hip_device)
    ms, vs = torch.zeros_like(ps_d), torch.zeros_like(ps_d)
    mw, vw = torch.zeros_like(pw_d), torch.zeros_like(pw_d)
    rms, rvs, rmw, rvw = (torch.zeros_like(t) for t in (p_s, p_s, p_w, p_w))
    c = coef.item()
    for t in range(1, 4):
        ops.adam_dense(cfg, ps_d, ms, vs, small.to(hip_device))
        ops.adam_rows(cfg, pw_d, mw, vw, rg)
        ops.counter_add(step, 1)
        R.adam_update(p_s, small * c, rms, rvs, t)
        R.adam_update(p_w, w1g * c, rmw, rvw, t)
    assert _maxrel(ps_d, p_s) < 1e-6 and _maxrel(pw_d, p_w) < 1e-6
    assert _maxrel(mw, rmw) < 1e-6 and _maxrel(vw, rvw) < 1e-5


def test_adam_flat_equals_split(ops, hip_device):
    """hvae_adam_flat (one launch over [W1t | pad | dense]) == hvae_adam_rows + hvae_adam_dense: bitwise over W1t
    and the pad; over the dense tail within a few ulp, since hvae_adam_dense (the eager drop-in step) follows torch's
    CPU arithmetic (correctly rounded sqrt and division, hvae_adam.h adam_elem_exact) while the fused trainer's flat
    launch keeps unfused products and the hardware square root and reciprocal (adam_elem)."""
    from hvae._lib import lib, ptr, stream_of
    from hvae import _lib
    g = torch.Generator().manual_seed(9)
    N, H, nd, off = 300, 64, 5003, 300 * 64 + 32
    X = synth_csr(20, N, seed=5)
    rg = ops.RowGradBuffers(N, H, int(X.nnz), hip_device)
    ops.w1_rowgrad(ops.csr_from_scipy(X, hip_device), torch.randn(20, H, generator=g).to(hip_device), rg)
    gd = torch.randn(nd, generator=g).to(hip_device)
    flat = torch.randn(off + nd, generator=g).to(hip_device)
    m, v = torch.randn_like(flat) * 0.1, torch.rand_like(flat) * 0.1
    step = torch.full((1,), 4, dtype=torch.int64, device=hip_device)
    coef = torch.full((1,), 0.7, device=hip_device)
    cfg = ops.adam_config(1e-3, (0.9, 0.999), 1e-8, 0.01, step, coef)
    p1, m1, v1 = flat.clone(), m.clone(), v.clone()
    ops.adam_rows(cfg, p1[: N * H].view(N, H), m1[: N * H].view(N, H), v1[: N * H].view(N, H), rg)
    ops.adam_dense(cfg, p1[off:], m1[off:], v1[off:], gd)
    p2, m2, v2 = flat.clone(), m.clone(), v.clone()
    _lib.check(lib().hvae_adam_flat(C.byref(cfg), ptr(p2), ptr(m2), ptr(v2), rg.ref, N, H, ptr(gd), off, nd,
                                    stream_of(p2)), "adam_flat")
    assert torch.equal(p1[:off], p2[:off]) and torch.equal(m1[:off], m2[:off]) and torch.equal(v1[:off], v2[:off])
    for a, b in ((p1, p2), (m1, m2), (v1, v2)):  # exact (fma-contracted, correctly rounded) vs fast: ~1 ulp
        assert torch.allclose(a[off:], b[off:], rtol=1e-6, atol=1e-7)


def test_clip_step_counters(ops, hip_device):
    """hvae_clip_grad_norm_step == hvae_clip_grad_norm + (snap = step; step += 1; boff += advance)."""
    from hvae import _lib
    from hvae._lib import lib, ptr, stream_of
    g = torch.Generator().manual_seed(6)
    small = torch.randn(70001, generator=g).to(hip_device)
    norm_a, coef_a = ops.clip_grad_norm(small, None, 1.0)
    norm, coef = torch.empty(1, device=hip_device), torch.empty(1, device=hip_device)
    step = torch.full((1,), 41, dtype=torch.int64, device=hip_device)
    snap = torch.zeros(1, dtype=torch.int64, device=hip_device)
    boff = torch.full((1,), 128, dtype=torch.int64, device=hip_device)
    ws = torch.empty(lib().hvae_clip_grad_norm_workspace(small.numel(), 0, 0), dtype=torch.uint8, device=hip_device)
    for _ in range(3):
        _lib.check(lib().hvae_clip_grad_norm_step(ptr(small), small.numel(), None, 0, 1.0, ptr(norm), ptr(coef),
                                                  ptr(step), ptr(snap), ptr(boff), 64, ptr(ws), ws.numel(),
                                                  stream_of(small)), "clip_step")
    assert torch.equal(norm, norm_a) and torch.equal(coef, coef_a)
    assert (int(step.item()), int(snap.item()), int(boff.item())) == (44, 43, 128 + 3 * 64)


@pytest.mark.parametrize("nb,N,lam,hot", [(40, 300, 5.0, 0), (64, 12101, 3.0, 40), (300, 2000, 8.0, 100), (5000, 500, 2.0, 4500),
                                         (40000, 3000, 1.0, 3000), (40000, 3000, 1.0, 6000),
                                         # catalogs past the one-block scan: the look-back scan over 4096-item blocks
                                         (4096, 100000, 15.0, 300), (2000, 1000003, 15.0, 0)])
def test_rowgrad_plan_apply_segments(ops, hip_device, nb, N, lam, hot):
    """Segments of every sort path (wave <= 64; bitmap rank for nb <= 32768; beyond that block bitonic
    <= 4096 and selection): plan + apply == dense reference, bitwise == the one-call form, and bitwise
    reproducible; contributions end sorted by batch row within each segment."""
    import scipy.sparse as sp
    from hvae._lib import lib, ptr, stream_of
    from hvae import _lib
    X = synth_csr(nb, N, lam=lam, seed=nb)
    if hot:  # item 0 in the first `hot` rows -> one long segment
        X = X.tolil()
        X[:hot, 0] = 1.0
        X = sp.csr_matrix(X)
    H = 128
    g = torch.Generator().manual_seed(1)
    da = torch.randn(nb, H, generator=g)
    xd = ops.csr_from_scipy(X, hip_device)
    dad = da.to(hip_device)
    rg = ops.RowGradBuffers(N, H, int(X.nnz), hip_device)
    ops.w1_rowgrad(xd, dad, rg)
    nu = int(rg.n_unique.item())
    one = rg.rows[:nu].clone()
    dense = torch.zeros(N, H, device=hip_device)
    ops.rowgrad_to_dense(rg, dense)
    ref = torch.as_tensor(np.asarray(X.T.astype(np.float64) @ da.double().numpy()))  # sparse: N may be 1M
    assert _maxrel(dense, ref) < 1e-5
    # slots in ascending item order, one per distinct item of the batch
    np.testing.assert_array_equal(rg.item_of[:nu].cpu().numpy(), np.unique(X.indices))
    st = stream_of(dad)
    _lib.check(lib().hvae_w1_rowgrad_plan(xd.ref, rg.ref, ptr(rg.ws), rg.ws.numel(), st), "plan")
    _lib.check(lib().hvae_w1_rowgrad_apply(ptr(dad), H, rg.ref, st), "apply")
    assert torch.equal(rg.rows[:nu], one)
    assert int(rg.cnt.abs().sum()) == 0 and int(rg.fill.abs().sum()) == 0
    seg = rg.seg_off[: nu + 1].cpu().numpy()
    crow = rg.contrib_row[: seg[-1]].cpu().numpy()
    cslot = rg.contrib_slot[: seg[-1]].cpu().numpy()
    for s_ in range(nu):
        assert np.all(np.diff(crow[seg[s_]:seg[s_ + 1]]) > 0)
        assert np.all(cslot[seg[s_]:seg[s_ + 1]] == s_)
    if hot:  # the long segment (its own sort path) against a float64 sum
        s0 = int((rg.item_of[:nu] == 0).nonzero()[0, 0])
        col0 = torch.as_tensor(X[:, 0].toarray().ravel(), dtype=torch.float64)
        assert _maxrel(rg.rows[s0], col0 @ da.double()) < 1e-5


# ------------------------------------------------------------------ eval ---
def test_candidates_rank_topk(ops, hip_device):
    N, D, R_ = 2000, 384, 50
    E = torch.as_tensor(synth_embeddings(N, D, seed=8))
    g = torch.Generator().manual_seed(8)
    U = torch.randn(R_, D, generator=g)
    cand = torch.stack([torch.randperm(N, generator=g)[:100] for _ in range(R_)]).int()
    Ed = E.to(hip_device)
    sc = ops.score_candidates(U.to(hip_device), torch.arange(R_, dtype=torch.int32, device=hip_device), Ed,
                              cand.to(hip_device))
    ref = (U.double() @ E.double().t()).gather(1, cand.long())
    assert _maxrel(sc, ref) < 1e-5
    rank = ops.rank_first(sc).cpu().numpy()
    s = sc.cpu().numpy()
    for r in range(R_):
        ranked = R.rank_candidates(s[r], np.arange(100))
        assert int(np.where(ranked == 0)[0][0]) == rank[r]
    # exact top-k on given scores, ties included (bit-exact indices)
    S = torch.randn(7, N, generator=g).round(decimals=1)  # many exact ties
    X = synth_csr(7, N, seed=9)
    idx, val = ops.topk(S.to(hip_device).clone(), 20, exclude=ops.csr_from_scipy(X, hip_device))
    for r in range(7):
        ref_idx = R.topk_exclude_seen(S[r].numpy(), X[r].indices, 20)
        np.testing.assert_array_equal(idx[r].cpu().numpy(), ref_idx)


def test_decoder_image_layout(ops, hip_device):
    """bf16 image = bf16(E) then the tile-transposed copy with items in the MFMA k order (tail items 0)."""
    N, D = 77, 64
    E = torch.as_tensor(synth_embeddings(N, D, seed=2))
    img = ops.decoder_image(E.to(hip_device))
    Eb = E.bfloat16()
    assert torch.equal(img.bf16.cpu(), Eb)
    off = (N * D * 2 + 255) // 256 * 256
    nt = (N + 31) // 32
    Et = img.buf[off: off + nt * D * 32 * 2].view(torch.bfloat16).view(nt, D, 32).cpu()
    pos_item = [16 * (p >> 4) + 4 * ((p >> 3) & 1) + 8 * ((p & 7) >> 2) + (p & 3) for p in range(32)]
    assert sorted(pos_item) == list(range(32))
    for t in range(nt):
        for p_, it in enumerate(pos_item):
            item = 32 * t + it
            want = Eb[item] if item < N else torch.zeros(D, dtype=torch.bfloat16)
            assert torch.equal(Et[t, :, p_], want)
