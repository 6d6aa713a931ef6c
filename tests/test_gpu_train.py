"""Fused train step (hvae/executor.py) vs the reference's own outputs (golden G2).

With the reference's dropout masks and reparameterisation noise injected, two
optimizer steps of the MI355X path must reproduce the reference's losses,
clip norm, pre-clip gradients, and parameters + Adam moments after step 2.
"""
import numpy as np
import pytest
import torch

from gen import TRAIN_CONFIGS, synth_csr, synth_embeddings
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu


def _maxrel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-30))


def _build(name, device, precision="fp32"):
    from hvae.executor import FusedTrainer
    from src.ml.model import HybridVAE
    c = TRAIN_CONFIGS[name]
    X = synth_csr(c["n_users"], c["n_items"], lam=c.get("lam", 3.0), seed=200 + c["seed"])
    E = synth_embeddings(c["n_items"], c["d"], seed=300 + c["seed"])
    torch.manual_seed(c["seed"])
    model = HybridVAE(c["n_items"], E, latent_dim=c["latent"], hidden_dims=c["hidden"], dropout=c["dropout"],
                      beta=c["beta"]).to(device)
    fused = FusedTrainer(model, device, lr=c["lr"], weight_decay=c.get("wd", 0.0), precision=precision,
                         use_graphs=False)
    data = fused.device_data(X, list(range(c["n_users"])))
    return c, X, E, model, fused, data


def _ext(golden, name, step, c, device):
    g = lambda k: torch.as_tensor(golden[f"g2{name}_s{step}_{k}"]).to(device)
    ext = {"enc_masks": [g(f"encmask{k}") for k in range(len(c["hidden"]))], "eps": g("eps")}
    if c["latent"] != c["d"]:
        ext["proj_mask"] = g("projmask")
    return ext


@pytest.mark.parametrize("name", sorted(TRAIN_CONFIGS))
def test_fused_step_matches_reference(golden, hip_device, name):
    from hvae import ops
    c, X, E, model, fused, data = _build(name, hip_device)
    B = c["n_users"]
    for step in (1, 2):
        loss3 = fused.step_batch(data, None, B, c["beta"], c["dropout"], train=True,
                                 ext=_ext(golden, name, step, c, hip_device))
        np.testing.assert_allclose(loss3.cpu().numpy(), golden[f"g2{name}_loss"][step - 1], rtol=2e-5, atol=1e-6)
        assert abs(fused.norm.item() - golden[f"g2{name}_norm"][step - 1]) <= 2e-5 * golden[f"g2{name}_norm"][step - 1]
        if step == 1:
            # pre-clip gradients (the reference's p.grad before clip_grad_norm_)
            for n in R.param_names(R.init_params(c["n_items"], E, c["latent"], c["hidden"], seed=c["seed"])):
                ref = golden[f"g2{name}_s1_grad_{n}"]
                if n == "encoder.0.weight":
                    bf = fused._bufs[(B, True)]
                    dense = torch.zeros(c["n_items"], c["hidden"][0], device=hip_device)
                    ops.rowgrad_to_dense(bf.rg, dense)
                    got = dense.t()
                elif n in ("fc_mu.weight", "fc_logvar.weight", "fc_mu.bias", "fc_logvar.bias"):
                    L = c["latent"]
                    Wg, bg = fused.gW_heads, fused.gb_heads
                    got = {"fc_mu.weight": Wg[:L], "fc_logvar.weight": Wg[L:], "fc_mu.bias": bg[:L],
                           "fc_logvar.bias": bg[L:]}[n]
                else:
                    got = fused.G[n]
                assert _maxrel(got, ref) < 2e-5, n
    params = dict(model.named_parameters())
    opt_m = {}
    for n, p in params.items():
        # Adam maps near-zero gradients to O(lr) steps: compare params relative to their magnitude
        assert _maxrel(p, golden[f"g2{name}_s2_param_{n}"]) < 5e-4, n
    lay = fused.layout
    for n in params:
        if n == "encoder.0.weight":
            m, v = fused.m_w1t.t(), fused.v_w1t.t()
        else:
            m, v = lay.view(fused.m, n), lay.view(fused.v, n)
        assert _maxrel(m, golden[f"g2{name}_s2_m_{n}"]) < 5e-5, n
        assert _maxrel(v, golden[f"g2{name}_s2_v_{n}"]) < 5e-5, n


@pytest.mark.parametrize("name", ["A", "C"])
def test_fused_step_bf16_decoder(golden, hip_device, name):
    """bf16 decoder MFMA: same step, looser tolerance (scores carry bf16 rounding of u and E)."""
    c, X, E, model, fused, data = _build(name, hip_device, precision="bf16")
    if fused.precision != "bf16":
        pytest.skip("no bf16 decoder for this d")
    B = c["n_users"]
    loss3 = fused.step_batch(data, None, B, c["beta"], c["dropout"], train=True,
                             ext=_ext(golden, name, 1, c, hip_device))
    np.testing.assert_allclose(loss3.cpu().numpy(), golden[f"g2{name}_loss"][0], rtol=2e-3)
    assert abs(fused.norm.item() - golden[f"g2{name}_norm"][0]) <= 1e-2 * golden[f"g2{name}_norm"][0]


def test_graph_replay_is_bitwise_eager(hip_device):
    """A hipGraph epoch reproduces the eager epoch bit for bit (same Philox streams, same kernels)."""
    from hvae.executor import ConstBeta, FusedTrainer
    from src.ml.model import HybridVAE
    X = synth_csr(300, 500, seed=3)
    E = synth_embeddings(500, 128, seed=4)
    outs = []
    for graphs in (False, True):
        torch.manual_seed(0)
        model = HybridVAE(500, E, latent_dim=64, hidden_dims=[128], dropout=0.3, beta=0.2).to(hip_device)
        fused = FusedTrainer(model, hip_device, precision="bf16", seed=1234, use_graphs=graphs)
        data = fused.device_data(X, list(range(300)))
        gen = torch.Generator().manual_seed(5)
        m1 = fused.run_epoch(data, 64, True, ConstBeta(0.2), 0.3, generator=gen)
        m2 = fused.run_epoch(data, 64, True, ConstBeta(0.2), 0.3, generator=gen)
        v = fused.run_epoch(data, 64, False, ConstBeta(0.2), 0.3)
        outs.append((m1, m2, v, fused.flat.clone()))
    (a1, a2, av, af), (b1, b2, bv, bf_) = outs
    assert a1 == b1 and a2 == b2 and av == bv
    assert torch.equal(af, bf_)
    assert a2["total_loss"] < a1["total_loss"]  # it learns


@pytest.mark.parametrize("wd,plan_side", [(0.0, False), (0.01, False), (0.01, True)])
def test_lazy_adam_is_bitwise_dense(hip_device, wd, plan_side, monkeypatch):
    """Exact lazy Adam (rows outside a batch replay their g = 0 steps when next read) leaves parameters and
    moments bitwise equal to torch's every-row update, over graph-replayed epochs with a short tail batch.
    plan_side: the W1-gradient plan on its own stream and the catch-up from the CSR entries
    (hvae_adam_lazy_catchup_csr), the large-batch configuration, forced at B = 32."""
    monkeypatch.setenv("HVAE_PLAN_SIDE_MIN_BATCH", "1" if plan_side else "1000000")
    from hvae.executor import ConstBeta, FusedTrainer
    from src.ml.model import HybridVAE
    X = synth_csr(290, 700, seed=13)
    E = synth_embeddings(700, 128, seed=14)
    outs = []
    for lazy in (False, True):
        torch.manual_seed(0)
        model = HybridVAE(700, E, latent_dim=64, hidden_dims=[128], dropout=0.3, beta=0.2).to(hip_device)
        fused = FusedTrainer(model, hip_device, weight_decay=wd, precision="bf16", seed=77, use_graphs=True)
        fused.lazy_adam = lazy
        data = fused.device_data(X, list(range(290)))
        gen = torch.Generator().manual_seed(6)
        r = [fused.run_epoch(data, 32, True, ConstBeta(0.2), 0.3, generator=gen) for _ in range(3)]
        v = fused.run_epoch(data, 32, False, ConstBeta(0.2), 0.3)
        outs.append((r, v, fused.flat.clone(), fused.m.clone(), fused.v.clone()))
    (ra, va, fa, ma, sa), (rb, vb, fb, mb, sb) = outs
    assert ra == rb and va == vb
    assert torch.equal(fa, fb) and torch.equal(ma, mb) and torch.equal(sa, sb)
