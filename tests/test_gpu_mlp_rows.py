"""The row-parallel latent / projection MLP (hvae_mlp_fwd_rows / hvae_mlp_bwd_rows / hvae_gemm_f32_multi).

Against float64 torch statements of model.py's fc_mu / fc_logvar, reparameterize and projection layers and
their autograd (explicit eps and dropout multipliers), against the unfused GEMM + reparam kernels on the
Philox path (the same noise and masks), and the whole train step with the row path on and off.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from gen import synth_csr, synth_embeddings

pytestmark = pytest.mark.gpu


def _maxrel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-30))


def _setup(B, H, L, D, dev, seed):
    g = torch.Generator().manual_seed(seed)
    t = dict(
        h=torch.randn(B, H, generator=g),
        Wh=torch.randn(2 * L, H, generator=g) / H ** 0.5, bh=torch.randn(2 * L, generator=g) * 0.1,
        Wa=torch.randn(D, L, generator=g) / L ** 0.5, ba=torch.randn(D, generator=g) * 0.1,
        Wb=torch.randn(D, D, generator=g) / D ** 0.5, bb=torch.randn(D, generator=g) * 0.1,
        eps=torch.randn(B, L, generator=g), mult=(torch.rand(B, D, generator=g) >= 0.3).float() / 0.7,
        dU=torch.randn(B, D, generator=g) * 0.01)
    d = {k: v.to(dev) for k, v in t.items()}
    out = dict(heads=torch.empty(B, 2 * L, device=dev), z=torch.empty(B, L, device=dev),
               eps_o=torch.empty(B, L, device=dev), kl=torch.empty(B, device=dev), p1=torch.empty(B, D, device=dev),
               q=torch.empty(B, D, device=dev), u=torch.empty(B, D, device=dev), dp1=torch.empty(B, D, device=dev),
               dheads=torch.empty(B, 2 * L, device=dev), dh=torch.empty(B, H, device=dev))
    return t, d, out


def _args(B, H, L, D, d, out, train, p_drop, explicit, seed=9, step=None):
    from hvae import _lib
    from hvae._lib import ptr
    return _lib.MlpRows(
        nb=B, H=H, L=L, D=D, W_heads=ptr(d["Wh"]), b_heads=ptr(d["bh"]), W_a=ptr(d["Wa"]), b_a=ptr(d["ba"]),
        W_b=ptr(d["Wb"]), b_b=ptr(d["bb"]), train=int(train), p_drop=p_drop,
        drop_mult=ptr(d["mult"]) if explicit else None, eps_in=ptr(d["eps"]) if explicit else None, seed=seed,
        step_dev=ptr(step), h=ptr(d["h"]), heads=ptr(out["heads"]), z=ptr(out["z"]), eps=ptr(out["eps_o"]),
        kl_rows=ptr(out["kl"]), p1=ptr(out["p1"]), q=ptr(out["q"]), u=ptr(out["u"]), dU=ptr(d["dU"]), ks=0.2 / B,
        ks_dev=None, dp1=ptr(out["dp1"]), dheads=ptr(out["dheads"]), dh=ptr(out["dh"]))


@pytest.mark.parametrize("B,H,L,D", [(1, 512, 128, 384), (7, 256, 64, 384), (64, 512, 128, 384),
                                     (129, 512, 128, 384), (300, 128, 64, 128), (513, 512, 128, 768),
                                     (1024, 512, 128, 384), (64, 512, 128, 768), (33, 96, 32, 64)])
@pytest.mark.parametrize("train", [True, False])
def test_mlp_rows_vs_float64(hip_device, B, H, L, D, train):
    from hvae._lib import GemmDesc, Epilogue, check, lib, ptr
    from hvae import _lib
    t, d, out = _setup(B, H, L, D, hip_device, B * 31 + D)
    a = _args(B, H, L, D, d, out, train, 0.3, explicit=True)
    check(lib().hvae_mlp_fwd_rows(C.byref(a), None), "mlp_fwd_rows")
    check(lib().hvae_mlp_bwd_rows(C.byref(a), None), "mlp_bwd_rows")
    # float64 reference with autograd (model.py's layers)
    T = {k: v.double().requires_grad_(k in ("h",)) for k, v in t.items()}
    heads = T["h"] @ T["Wh"].t() + T["bh"]
    mu, lv = heads[:, :L], heads[:, L:]
    mu.retain_grad()
    lv.retain_grad()
    z = mu + T["eps"] * torch.exp(0.5 * lv) if train else mu
    kl_rows = -0.5 * (1 + lv - mu ** 2 - lv.exp()).sum(1)
    p1 = z @ T["Wa"].t() + T["ba"]
    q = torch.nn.functional.gelu(p1) * (T["mult"] if train else 1.0)
    u = q @ T["Wb"].t() + T["bb"]
    for name, got, ref in [("heads", out["heads"], heads), ("z", out["z"], z), ("kl", out["kl"], kl_rows),
                           ("p1", out["p1"], p1), ("q", out["q"], q), ("u", out["u"], u)]:
        assert _maxrel(got, ref) < 2e-6 * max(1.0, (H / 64) ** 0.5), name
    if train:
        assert torch.equal(out["eps_o"].cpu(), t["eps"])
    # backward: the loss u . dU + (beta / B) sum kl_rows
    p1.retain_grad()
    (u * T["dU"]).sum().add((0.2 / B) * kl_rows.sum()).backward()
    assert _maxrel(out["dp1"], p1.grad) < 2e-6 * max(1.0, (D / 64) ** 0.5)
    assert _maxrel(out["dheads"][:, :L], mu.grad) < 5e-6 and _maxrel(out["dheads"][:, L:], lv.grad) < 5e-6
    assert _maxrel(out["dh"], T["h"].grad) < 5e-6
    # the three weight gradients (+ bias gradients) in one launch
    gWb, gWa, gWh = (torch.empty(D, D, device=hip_device), torch.empty(D, L, device=hip_device),
                     torch.empty(2 * L, H, device=hip_device))
    gbb, gba, gbh = (torch.empty(D, device=hip_device), torch.empty(D, device=hip_device),
                     torch.empty(2 * L, device=hip_device))
    keep = []

    def desc(M, N, A, lda, Bm, ldb, Cm, ldc, rs):
        e = Epilogue(_lib.EPI_NONE, None, None, None, 0.0, None, 0, None, 0, 0, ptr(rs))
        keep.append(e)
        return GemmDesc(1, 0, M, N, B, 1.0, ptr(A), lda, ptr(Bm), ldb, 0.0, ptr(Cm), ldc, C.pointer(e), None, 0)
    ds = (GemmDesc * 3)(desc(D, D, d["dU"], D, out["q"], D, gWb, D, gbb),
                        desc(D, L, out["dp1"], D, out["z"], L, gWa, L, gba),
                        desc(2 * L, H, out["dheads"], 2 * L, d["h"], H, gWh, H, gbh))
    check(lib().hvae_gemm_f32_multi(ds, 3, None), "gemm_multi")
    dU64, dp164, dh64 = T["dU"], p1.grad, torch.cat([mu.grad, lv.grad], 1)
    assert _maxrel(gWb, dU64.t() @ q.detach()) < 1e-5 and _maxrel(gbb, dU64.sum(0)) < 1e-5
    assert _maxrel(gWa, dp164.t() @ z.detach()) < 1e-5 and _maxrel(gba, dp164.sum(0)) < 1e-5
    assert _maxrel(gWh, dh64.t() @ T["h"].detach()) < 1e-5 and _maxrel(gbh, dh64.sum(0)) < 1e-5


def test_mlp_rows_philox_matches_unfused(hip_device):
    """Without explicit noise / masks the row kernel draws the same Philox streams as hvae_reparam_kl_fwd and
    the BIAS_GELU_DROP epilogue (tag 0x200), so eps is bitwise equal and the dropout pattern identical."""
    from hvae import _lib, ops
    from hvae._lib import check, lib
    B, H, L, D = 64, 512, 128, 384
    t, d, out = _setup(B, H, L, D, hip_device, 3)
    step = torch.tensor([5], dtype=torch.int64, device=hip_device)
    a = _args(B, H, L, D, d, out, True, 0.3, explicit=False, seed=1234, step=step)
    check(lib().hvae_mlp_fwd_rows(C.byref(a), None), "mlp_fwd_rows")
    heads = ops.gemm(d["h"], d["Wh"].t(), epi=ops.epilogue(_lib.EPI_BIAS, bias=d["bh"]))
    z, eps, kl = ops.reparam_kl_fwd(heads[:, :L], heads[:, L:], True, 1234, step=step)
    pre = torch.empty(B, D, device=hip_device)
    q = ops.gemm(z, d["Wa"].t(), epi=ops.epilogue(_lib.EPI_BIAS_GELU_DROP, bias=d["ba"], pre_out=pre, p_drop=0.3,
                                                  seed=1234, step=step, tag=_lib.TAG_PROJ_DROP, train=True))
    assert torch.equal(out["eps_o"], eps)
    assert torch.equal(out["q"] == 0, q == 0)
    assert _maxrel(out["heads"], heads) < 1e-6 and _maxrel(out["z"], z) < 1e-6 and _maxrel(out["q"], q) < 1e-6
    assert _maxrel(out["kl"], kl) < 1e-6


@pytest.mark.parametrize("B", [64, 200])
def test_train_step_mlp_rows_equals_gemm_chain(hip_device, B):
    """The fused trainer with the row-parallel MLP and with the GEMM chain: the same losses and parameters up to
    fp32 summation order, over graph-replayed epochs."""
    from hvae.executor import ConstBeta, FusedTrainer
    from src.ml.model import HybridVAE
    X = synth_csr(600, 900, seed=21)
    E = synth_embeddings(900, 384, seed=22)
    outs = []
    for rows in (False, True):
        torch.manual_seed(0)
        model = HybridVAE(900, E, latent_dim=128, hidden_dims=[512], dropout=0.3, beta=0.2).to(hip_device)
        fused = FusedTrainer(model, hip_device, precision="fp32", seed=55, use_graphs=True)
        fused.mlp_rows = rows
        assert fused._mlp_rows_ok(B) == rows
        data = fused.device_data(X, list(range(600)))
        gen = torch.Generator().manual_seed(7)
        r = [fused.run_epoch(data, B, True, ConstBeta(0.2), 0.3, generator=gen) for _ in range(2)]
        v = fused.run_epoch(data, B, False, ConstBeta(0.2), 0.3)
        outs.append((r, v, fused.flat.cpu().numpy()))
    (ra, va, fa), (rb, vb, fb) = outs
    for ea, eb in zip(ra + [va], rb + [vb]):
        for k in ea:
            assert abs(ea[k] - eb[k]) <= 1e-5 * max(abs(eb[k]), 1e-3), (k, ea[k], eb[k])
    # Adam can turn a rounding-level gradient difference into a +-lr step on a near-zero gradient
    assert float(np.abs(fa.astype(np.float64) - fb).max()) <= 2 * 2 * 1e-3


@pytest.mark.parametrize("nb,N,lam", [(64, 12101, 3.0), (7, 300, 5.0), (300, 2000, 8.0)])
def test_plan_block_in_mlp_launch_equals_plan(hip_device, nb, N, lam):
    """The W1 row-gradient plan run as the extra block of hvae_mlp_fwd_rows' launch writes exactly what
    hvae_w1_rowgrad_plan's one-block plan writes (slots, segments, sorted contributions), and the rows' outputs
    do not change."""
    from hvae import _lib, ops
    from hvae._lib import check, lib, ptr
    X = synth_csr(nb, N, lam=lam, seed=nb + 1)
    assert X.nnz <= _lib.PLAN_SMALL_CAP
    xd = ops.csr_from_scipy(X, hip_device)
    H, L, D = 512, 128, 384
    t, d, out = _setup(nb, H, L, D, hip_device, 5)
    outs = []
    for fused in (False, True):
        rg = ops.RowGradBuffers(N, H, int(X.nnz), hip_device)
        for tn in (rg.slot_of, rg.item_of, rg.seg_off, rg.contrib_row, rg.contrib_slot):
            tn.fill_(-7)
        rg.contrib_val.fill_(-7.0)
        a = _args(nb, H, L, D, d, out, True, 0.3, explicit=True)
        if fused:
            a.plan_x, a.plan_rg = C.pointer(xd.struct), C.pointer(rg.struct)
        else:
            check(lib().hvae_w1_rowgrad_plan(xd.ref, rg.ref, ptr(rg.ws), rg.ws.numel(), None), "plan")
        check(lib().hvae_mlp_fwd_rows(C.byref(a), None), "mlp_fwd_rows")
        torch.cuda.synchronize()
        nu = int(rg.n_unique.item())
        T = int(X.nnz)
        items = torch.as_tensor(np.unique(X.indices), dtype=torch.long, device=hip_device)
        outs.append((nu, rg.item_of[:nu].clone(), rg.seg_off[:nu + 1].clone(), rg.contrib_row[:T].clone(),
                     rg.contrib_val[:T].clone(), rg.contrib_slot[:T].clone(), rg.slot_of[items].clone(),
                     out["u"].clone()))
    (a0, *r0), (a1, *r1) = outs
    assert a0 == a1
    for x0, x1 in zip(r0, r1):
        assert torch.equal(x0, x1)


@pytest.mark.parametrize("B,H,train,explicit", [(64, 512, True, False), (7, 256, True, True), (300, 512, False, False),
                                                (1024, 512, True, False), (33, 96, True, False)])
def test_mlp_bwd_fused_layernorm_equals_ln_bwd(hip_device, B, H, train, explicit):
    """The LayerNorm -> GELU -> Dropout backward fused into hvae_mlp_bwd_rows gives hvae_ln_gelu_drop_bwd's da bit
    for bit (same per-row arithmetic and lane order) and its column sums (d_ln_w, d_ln_b, d_bias) to fp32 rounding
    (blocks of other row counts)."""
    from hvae import _lib, ops
    from hvae._lib import check, lib, ptr
    L, D = 128 if H >= 256 else 32, 384 if H >= 256 else 64
    t, d, out = _setup(B, H, L, D, hip_device, 11)
    g = torch.Generator().manual_seed(12)
    xhat = torch.randn(B, H, generator=g).to(hip_device)
    rstd = (torch.rand(B, generator=g) + 0.5).to(hip_device)
    ln_w = (torch.randn(H, generator=g) * 0.2 + 1).to(hip_device)
    ln_b = (torch.randn(H, generator=g) * 0.1).to(hip_device)
    emult = ((torch.rand(B, H, generator=g) >= 0.3).float() / 0.7).to(hip_device) if explicit else None
    step = torch.tensor([3], dtype=torch.int64, device=hip_device)
    a = _args(B, H, L, D, d, out, train, 0.3, explicit=True, seed=77, step=step)
    check(lib().hvae_mlp_fwd_rows(C.byref(a), None), "mlp_fwd_rows")
    da, dw, db, dbias = (torch.full((B, H), 7.0, device=hip_device), torch.empty(H, device=hip_device),
                         torch.empty(H, device=hip_device), torch.empty(H, device=hip_device))
    ws = torch.empty(max(int(lib().hvae_mlp_bwd_rows_workspace(B, H)), 256), dtype=torch.uint8, device=hip_device)
    a.ln_w, a.ln_b, a.xhat, a.rstd, a.enc_drop_mult, a.enc_layer = (ptr(ln_w), ptr(ln_b), ptr(xhat), ptr(rstd),
                                                                      ptr(emult), 0)
    a.da, a.d_ln_w, a.d_ln_b, a.d_bias, a.ws, a.ws_bytes = ptr(da), ptr(dw), ptr(db), ptr(dbias), ptr(ws), ws.numel()
    check(lib().hvae_mlp_bwd_rows(C.byref(a), None), "mlp_bwd_rows")
    da2, dw2, db2, dbias2 = ops.ln_gelu_drop_bwd(out["dh"], xhat, rstd, ln_w, ln_b, 0.3, train, 77, 0, step=step,
                                                 drop_mult=emult, want_dbias=True)
    assert torch.equal(da, da2)
    assert _maxrel(dw, dw2) < 1e-5 and _maxrel(db, db2) < 1e-5 and _maxrel(dbias, dbias2) < 1e-5


@pytest.mark.parametrize("B", [64, 300])
def test_mlp_bwd_deferred_layernorm_columns(hip_device, B):
    """With d_ln_w = d_ln_b = d_bias = NULL hvae_mlp_bwd_rows leaves its per-block column sums in ws
    ([hvae_mlp_rows_blocks(B)][3][H]) and hvae_gemm_f32_multi finishes them (partials^T x ones), as the fused
    trainer does: da bitwise the in-launch reduction's, the three column sums to fp32 rounding of its block-order
    sums."""
    from hvae import _lib
    from hvae._lib import GemmDesc, check, lib, ptr
    H, L, D = 512, 128, 384
    t, d, out = _setup(B, H, L, D, hip_device, 13)
    g = torch.Generator().manual_seed(14)
    xhat = torch.randn(B, H, generator=g).to(hip_device)
    rstd = (torch.rand(B, generator=g) + 0.5).to(hip_device)
    ln_w = (torch.randn(H, generator=g) * 0.2 + 1).to(hip_device)
    ln_b = (torch.randn(H, generator=g) * 0.1).to(hip_device)
    step = torch.tensor([4], dtype=torch.int64, device=hip_device)
    res = []
    for deferred in (False, True):
        a = _args(B, H, L, D, d, out, True, 0.3, explicit=True, seed=78, step=step)
        check(lib().hvae_mlp_fwd_rows(C.byref(a), None), "mlp_fwd_rows")
        da, dw, db, dbias = (torch.full((B, H), 7.0, device=hip_device), torch.empty(H, device=hip_device),
                             torch.empty(H, device=hip_device), torch.empty(H, device=hip_device))
        ws = torch.empty(max(int(lib().hvae_mlp_bwd_rows_workspace(B, H)), 256), dtype=torch.uint8, device=hip_device)
        a.ln_w, a.ln_b, a.xhat, a.rstd, a.enc_drop_mult, a.enc_layer = ptr(ln_w), ptr(ln_b), ptr(xhat), ptr(rstd), None, 0
        a.da, a.ws, a.ws_bytes = ptr(da), ptr(ws), ws.numel()
        if deferred:
            a.d_ln_w = a.d_ln_b = a.d_bias = None
        else:
            a.d_ln_w, a.d_ln_b, a.d_bias = ptr(dw), ptr(db), ptr(dbias)
        check(lib().hvae_mlp_bwd_rows(C.byref(a), None), "mlp_bwd_rows")
        if deferred:
            nblk = int(lib().hvae_mlp_rows_blocks(B))
            ones = torch.ones(nblk, device=hip_device)
            descs = (GemmDesc * 3)(*[GemmDesc(1, 0, H, 1, nblk, 1.0, ptr(ws) + 4 * k * H, 3 * H, ptr(ones), 1, 0.0,
                                              ptr(o), 1, None, None, 0) for k, o in enumerate((dw, db, dbias))])
            check(lib().hvae_gemm_f32_multi(descs, 3, None), "gemm_multi")
        res.append((da.clone(), dw.clone(), db.clone(), dbias.clone()))
    (da0, dw0, db0, dbias0), (da1, dw1, db1, dbias1) = res
    assert torch.equal(da0, da1)
    assert _maxrel(dw1, dw0) < 1e-5 and _maxrel(db1, db0) < 1e-5 and _maxrel(dbias1, dbias0) < 1e-5
