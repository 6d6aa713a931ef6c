"""fp8 decoder (BASELINE configs[4]): block-scaled e4m3 MFMA sweep through the C ABI.

Parity is stated against two references:
  * the same math on the QUANTISED operands in fp64 (E8 = e4m3(E 2^ke) 2^-ke, u8 = e4m3(u 2^ku) 2^-ku, the
    exponents from max |E| and max |u_b| as hvae_decoder.hip picks them): lse must agree to fp32 accumulation
    error (rel 2e-4); O additionally carries the e4m3 rounding of P (3 mantissa bits, per-user per-64-item
    block exponent): every element must lie inside the worst-case envelope of that rounding,
    |O - O_ref| <= 2^-4 (softmax(S) |E8|) + 2^-11 max|E8| (normal terms rounded to half an ulp, 2^-4 of
    themselves; subnormal q < 2^-6 of a block whose max is >= 2^7 at most 2^-17 of the block max each);
  * the reference's fp32 scores (model.py:198, 281) with unquantised E and U: the fp8 input rounding itself,
    loss rows rel 2e-2, d(u) max-rel 1e-1 (reported, not a kernel-correctness bar).
"""
import math

import numpy as np
import pytest
import torch

from gen import synth_csr, synth_embeddings

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(hip_device):
    from hvae import _lib, ops
    if not ops.decoder_supported(_lib.HVAE_FP8, 384):
        pytest.fail("libhvae has no fp8 decoder for D = 384")
    return ops


def _maxrel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-30))


def _pow2_exp(amax: torch.Tensor) -> torch.Tensor:
    """k with max |x 2^k| <= 256, as the kernels choose it (8 - frexp exponent; 0 for an all-zero row)."""
    _, e = torch.frexp(amax)
    return torch.where(amax > 0, torch.clamp(8 - e, max=127), torch.zeros_like(e))


def _q(x: torch.Tensor, k: torch.Tensor) -> torch.Tensor:
    s = torch.ldexp(torch.ones_like(x), k.to(x.dtype) if k.dim() else k.expand_as(x).to(x.dtype))
    return (x * s).to(torch.float8_e4m3fn).float() / s


def _quantised(E: torch.Tensor, U: torch.Tensor):
    ke = _pow2_exp(E.abs().max())
    ku = _pow2_exp(U.abs().amax(1, keepdim=True))
    return _q(E, ke), _q(U, ku), int(ke)


def _o_envelope(S: torch.Tensor, Eq: torch.Tensor) -> torch.Tensor:
    """Worst-case |O - O_ref| from rounding P to e4m3 with a per-(user, 64-item tile) power-of-two scale."""
    return 2.0 ** -4 * (torch.softmax(S, 1) @ Eq.double().abs()) + 2.0 ** -11 * Eq.abs().max().item()


def _image(ops, E):
    from hvae import _lib
    return ops.decoder_image(E, _lib.HVAE_FP8)


def _sw(D, it):
    """hvae_decoder.hip f8_sw: XOR swizzle of the 16-B chunks of item row `it` of a tile."""
    if D % 256 == 0:
        return ((it & 1) << 1) | (((it >> 1) & 1) << 2) | (((it >> 3) & 1) << 3) | ((it >> 2) & 1)
    return ((it >> 1) & 1) | ((((it >> 1) ^ (it >> 2)) & 1) << 1) | (((it >> 3) & 1) << 2)


@pytest.mark.parametrize("N,D", [(150, 128), (70, 768), (65, 384)])
def test_fp8_image_layout(ops, hip_device, N, D):
    """bf16 part == bf16(E); e4m3 tiles [64][D] with swizzled chunks == torch's e4m3 of E 2^ke; ke at the tail."""
    E = torch.as_tensor(synth_embeddings(N, D, seed=4)) * 3.0
    img = _image(ops, E.to(hip_device))
    assert torch.equal(img.bf16.cpu(), E.bfloat16())
    off = (N * D * 2 + 255) // 256 * 256
    nt = (N + 63) // 64
    raw = img.buf.cpu()
    tail = off + nt * 64 * D
    ke = int(raw[tail: tail + 4].view(torch.int32)[0])
    assert ke == int(_pow2_exp(E.abs().max()))
    E8 = torch.zeros(nt * 64, D, dtype=torch.float8_e4m3fn)
    E8[:N] = (E * 2.0 ** ke).to(torch.float8_e4m3fn)
    want = torch.empty(nt * 64 * D, dtype=torch.uint8)
    E8u = E8.view(torch.uint8)
    for item in range(nt * 64):
        t, it = divmod(item, 64)
        for ch in range(D // 16):
            o = t * 64 * D + it * D + 16 * (ch ^ _sw(D, it))
            want[o: o + 16] = E8u[item, 16 * ch: 16 * ch + 16]
    assert torch.equal(raw[off: tail], want)


@pytest.mark.parametrize("nb,N,D", [(3, 50, 384), (64, 890, 384), (200, 12101, 384), (130, 1000, 128),
                                    (300, 5000, 256), (520, 20011, 384), (64, 2000, 768), (300, 5001, 768),
                                    (7, 100, 768)])
def test_decoder_fp8(ops, hip_device, nb, N, D):
    """The fp8 sweep (k_dec_fp8; at d = 768 k_dec5_f8, producer / consumer waves) against float64 on the quantised operands.
    (k_dec4_f8, the version-4 structure it tied with, runs on the A/B variant: tests/ab_checks.py.)"""
    E = torch.as_tensor(synth_embeddings(N, D, seed=N))
    g = torch.Generator().manual_seed(nb)
    U = torch.randn(nb, D, generator=g) * 3.0
    img = _image(ops, E.to(hip_device))
    enorm = ops.row_norm_max(img)
    lse, O = ops.decoder_fwd(U.to(hip_device), img, enorm)
    Eq, Uq, _ = _quantised(E, U)
    S = Uq.double() @ Eq.double().t()
    lse_ref = torch.logsumexp(S, 1)
    O_ref = torch.softmax(S, 1) @ Eq.double()
    assert torch.isfinite(lse).all() and torch.isfinite(O).all()
    assert (lse.double().cpu() - lse_ref).abs().max() < 2e-4 * max(1.0, lse_ref.abs().max().item())
    err = (O.double().cpu() - O_ref).abs()
    assert (err <= _o_envelope(S, Eq)).all(), float((err / _o_envelope(S, Eq)).max())
    print(f"fp8 O max-rel {_maxrel(O, O_ref):.4f}, envelope use {float((err / _o_envelope(S, Eq)).max()):.3f}")
    lse2, _ = ops.decoder_fwd(U.to(hip_device), img, enorm, with_o=False)
    assert torch.allclose(lse2, lse, rtol=0, atol=1e-5)


def test_decoder_fp8_large_norm_fixup(ops, hip_device):
    """|u| in the hundreds: the fixed offset flags underflowing users, the finalize recomputes them exactly."""
    N, D = 4000, 128
    E = torch.as_tensor(synth_embeddings(N, D, seed=9))
    g = torch.Generator().manual_seed(1)
    U = torch.randn(8, D, generator=g)
    U = U / U.norm(dim=1, keepdim=True) * torch.tensor([1, 10, 50, 100, 200, 400, 800, 1500.0])[:, None]
    img = _image(ops, E.to(hip_device))
    lse, O = ops.decoder_fwd(U.to(hip_device), img, ops.row_norm_max(img))
    assert torch.isfinite(lse).all() and torch.isfinite(O).all()
    S = U.double() @ E.double().t()
    ref = torch.logsumexp(S, 1)
    assert ((lse.double().cpu() - ref).abs() / ref.abs().clamp(min=1)).max() < 2e-2


@pytest.mark.parametrize("nb,N,D", [(40, 700, 384), (64, 12101, 384), (5, 3000, 128), (300, 9000, 256),
                                    (130, 4000, 768)])
def test_decoder_train_fused_fp8(ops, hip_device, nb, N, D):
    """Fused sweep + finalize == decoder_fwd + decoder_bwd (bitwise), and == autograd on the quantised scores."""
    X = synth_csr(nb, N, lam=5.0, seed=nb + N)
    x = torch.as_tensor(X.toarray(), dtype=torch.float32)
    E = torch.as_tensor(synth_embeddings(N, D, seed=3))
    g = torch.Generator().manual_seed(5)
    U = torch.randn(nb, D, generator=g) * 2
    xd = ops.csr_from_scipy(X, hip_device)
    Ed, Ud = E.to(hip_device), U.to(hip_device)
    img = _image(ops, Ed)
    enorm = ops.row_norm_max(img)
    lse, O, rr, dU = ops.decoder_train(xd, Ud, img, enorm, Ed, 1.0 / nb, want_o=True)
    lse_b, O_b = ops.decoder_fwd(Ud, img, enorm)
    rr_b, dU_b = ops.decoder_bwd(xd, Ud, Ed, lse_b, O_b, 1.0 / nb)
    assert torch.equal(lse, lse_b) and torch.equal(rr, rr_b) and torch.equal(dU, dU_b) and torch.equal(O, O_b)
    # recon rows / d(u): finalize terms use fp32 E and u (sparse part exact), the sweep the quantised ones
    Eq, Uq, _ = _quantised(E, U)
    Sq = Uq.double() @ Eq.double().t()
    lse_q = torch.logsumexp(Sq, 1)
    xs = x.double()
    rr_q = xs.sum(1) * lse_q - (xs * (U.double() @ E.double().t())).sum(1)
    assert _maxrel(rr, rr_q) < 2e-3
    dU_q = (xs.sum(1, keepdim=True) * (torch.softmax(Sq, 1) @ Eq.double()) - xs @ E.double()) / nb
    env = xs.sum(1, keepdim=True) / nb * _o_envelope(Sq, Eq) + 1e-6 * dU_q.abs().max().item()
    assert ((dU.double().cpu() - dU_q).abs() <= env).all()
    # against the unquantised fp32 reference (the input rounding of fp8, reported bound)
    u_ = U.clone().requires_grad_(True)
    rr_t = -(x * torch.log_softmax(u_ @ E.t(), 1)).sum(1)
    rr_t.mean().backward()
    assert _maxrel(rr, rr_t) < 2e-2
    assert _maxrel(dU, u_.grad) < 1e-1


def test_fused_trainer_fp8_steps(hip_device):
    """FusedTrainer(precision='fp8') runs graph-captured epochs; its loss tracks the bf16 trainer's."""
    from hvae.executor import FusedTrainer
    from src.ml.model import HybridVAE
    n_users, n_items, d = 512, 3000, 384
    X = synth_csr(n_users, n_items, seed=11)
    E = synth_embeddings(n_items, d, seed=12)
    losses = {}
    for prec in ("bf16", "fp8"):
        torch.manual_seed(0)
        model = HybridVAE(n_items, E, latent_dim=128, hidden_dims=[512], dropout=0.3, beta=0.2).to(hip_device)
        fused = FusedTrainer(model, hip_device, precision=prec, seed=1234, use_graphs=True)
        assert fused.precision == prec
        data = fused.device_data(X, list(range(n_users)))
        hist = []
        for ep in range(3):
            m = fused.run_epoch(data, 64, True, lambda i: 0.2, 0.3, train=True,
                                generator=torch.Generator().manual_seed(ep))
            hist.append(m["total_loss"])
        losses[prec] = np.array(hist)
        assert np.isfinite(losses[prec]).all()
    assert losses["fp8"][-1] < losses["fp8"][0]
    np.testing.assert_allclose(losses["fp8"], losses["bf16"], rtol=2e-2)
