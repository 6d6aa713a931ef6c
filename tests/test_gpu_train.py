"""Fused train step (hvae/executor.py) vs the reference's own outputs (golden G2).

With the reference's dropout masks and reparameterisation noise injected, two
optimizer steps of the MI355X path must reproduce the reference's losses,
clip norm, pre-clip gradients, and parameters + Adam moments after step 2.
"""
import numpy as np
import pytest
import torch

from gen import EVAL_CONFIG, TRAIN_CONFIGS, synth_csr, synth_embeddings
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


def _step_errors(golden, hip_device, name, precision):
    """Two fused steps with the reference's masks and noise injected; the largest relative deviation from golden
    G2 of each compared quantity (losses, clip norm, pre-clip grads of step 1, params / m / v after step 2)."""
    from hvae import ops
    c, X, E, model, fused, data = _build(name, hip_device, precision)
    B = c["n_users"]
    err = {"loss": 0.0, "norm": 0.0}
    for step in (1, 2):
        loss3 = fused.step_batch(data, None, B, c["beta"], c["dropout"], train=True,
                                 ext=_ext(golden, name, step, c, hip_device))
        ref = np.asarray(golden[f"g2{name}_loss"][step - 1])
        err["loss"] = max(err["loss"], float(np.max(np.abs(loss3.cpu().numpy() - ref) / np.abs(ref))))
        nr = golden[f"g2{name}_norm"][step - 1]
        err["norm"] = max(err["norm"], abs(fused.norm.item() - nr) / nr)
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
                err[f"grad:{n}"] = _maxrel(got, ref)
    params = dict(model.named_parameters())
    lay = fused.layout
    for n, p in params.items():
        ref = golden[f"g2{name}_s2_param_{n}"]
        if precision == "fp32":  # params relative to their magnitude
            err[f"param:{n}"] = _maxrel(p, ref)
        else:
            # Adam's early steps are ~lr * sign(g): a gradient near 0 whose sign the decoder's rounding flips
            # moves its element by 2 lr (biases start at 0, so any max-relative bar fails on them); the bar is
            # on the RMS deviation in units of lr over the tensor
            dev = p.detach().double().cpu() - torch.as_tensor(ref).double()
            err[f"param:{n}"] = float(dev.pow(2).mean().sqrt()) / c["lr"]
        if n == "encoder.0.weight":
            m, v = fused.m_w1t.t(), fused.v_w1t.t()
        else:
            m, v = lay.view(fused.m, n), lay.view(fused.v, n)
        err[f"m:{n}"] = _maxrel(m, golden[f"g2{name}_s2_m_{n}"])
        err[f"v:{n}"] = _maxrel(v, golden[f"g2{name}_s2_v_{n}"])
    return err


def _check(err, tol, label):
    print(label, {k: f"{v:.2e}" for k, v in err.items()})
    bad = {k: v for k, v in err.items() if v > tol[k.split(":")[0]]}
    assert not bad, (label, bad)


# Bars per decoder precision: relative, max over elements, scaled by the reference tensor's max ("param" in
# low precision: RMS deviation in units of lr, see _step_errors). Measured on MI355X (profiles/r02_train_pins.log),
# max over configs A / C: bf16 loss 2e-4, norm 1.1e-3, grads 3.9e-3, m / v 4.1e-3; fp8 (A) loss 6.7e-4,
# norm 8e-3, grads 4.7e-2, m 8e-2, v 9.1e-2.
#   fp32: the fused kernels in exact fp32 (reduction order only);
#   bf16: S = u E^T from bf16-rounded u and E (2^-9 relative each) and P rounded to bf16 for O = P E;
#   fp8:  e4m3 u and E (2^-4 relative rounding) and P in e4m3 blocks: ~10x bf16's deviations.
STEP_TOL = {
    "fp32": {"loss": 2e-5, "norm": 2e-5, "grad": 2e-5, "param": 5e-4, "m": 5e-5, "v": 5e-5},
    "bf16": {"loss": 2e-3, "norm": 5e-3, "grad": 1e-2, "param": 0.15, "m": 1e-2, "v": 1.5e-2},
    "fp8": {"loss": 5e-3, "norm": 3e-2, "grad": 1.2e-1, "param": 0.6, "m": 2e-1, "v": 2.5e-1},
}


@pytest.mark.parametrize("name", sorted(TRAIN_CONFIGS))
def test_fused_step_matches_reference(golden, hip_device, name):
    _check(_step_errors(golden, hip_device, name, "fp32"), STEP_TOL["fp32"], f"fp32 {name}")


@pytest.mark.parametrize("name,precision", [("A", "bf16"), ("C", "bf16"), ("A", "fp8")])
def test_fused_step_low_precision_decoder(golden, hip_device, name, precision):
    """bf16 / fp8 decoder MFMA: the same two steps against golden G2 at the bars of STEP_TOL (production
    precisions; the whole train step, not only its losses)."""
    from hvae import ops, _lib
    d = TRAIN_CONFIGS[name]["d"]
    if not ops.decoder_supported(_lib.HVAE_BF16 if precision == "bf16" else _lib.HVAE_FP8, d):
        pytest.skip(f"no {precision} decoder for d = {d}")
    _check(_step_errors(golden, hip_device, name, precision), STEP_TOL[precision], f"{precision} {name}")


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp8"])
def test_validate_loss_matches_reference(golden, hip_device, precision):
    """VAETrainer.validate's per-batch loss (eval mode: z = mu, no dropout; reference src/ml/train.py:105-124,
    model.py:157-179) from the fused step against the reference's eval-mode loss terms on the G1 inputs."""
    from hvae.executor import FusedTrainer
    from src.ml.model import HybridVAE
    c = EVAL_CONFIG
    X = synth_csr(c["n_users"], c["n_items"], seed=100)
    E = synth_embeddings(c["n_items"], c["d"], seed=101)
    torch.manual_seed(c["seed"])
    model = HybridVAE(c["n_items"], E, latent_dim=c["latent"], hidden_dims=c["hidden"], dropout=0.3,
                      beta=c["beta"]).to(hip_device)
    fused = FusedTrainer(model, hip_device, precision=precision, use_graphs=False)
    data = fused.device_data(X, list(range(c["n_users"])))
    loss3 = fused.step_batch(data, None, c["n_users"], c["beta"], 0.3, train=False).cpu().numpy()
    ref = golden["g1_loss"]
    err = np.abs(loss3 - ref) / np.abs(ref)
    print(precision, "val loss rel err", err)
    assert np.all(err < STEP_TOL[precision]["loss"]), (loss3, ref)


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


@pytest.mark.parametrize("lazy_read", [True, False])
@pytest.mark.parametrize("wd,plan_side", [(0.0, False), (0.01, False), (0.01, True), (0.0, True)])
def test_lazy_adam_is_bitwise_dense(hip_device, wd, plan_side, lazy_read, monkeypatch):
    """Exact lazy Adam (rows outside a batch replay their g = 0 steps when next read) leaves parameters and
    moments bitwise equal to the every-row update, over graph-replayed epochs with a short tail batch.
    plan_side: the W1-gradient plan on its own stream and the catch-up from the CSR entries
    (hvae_adam_lazy_catchup_csr), the large-batch configuration, forced at B = 32 -- with wd = 0 its p-only
    replays (bits 24-29 of last_step) and the per-row slicing of small batches, with wd != 0 the full-store
    branch. lazy_read=False: the small-batch forward's CSR catch-up launch instead of the row-parallel encoder
    reading W1t through lazy Adam in registers (HVAE_ENC_LAZY_READ=0)."""
    monkeypatch.setenv("HVAE_PLAN_SIDE_MIN_BATCH", "1" if plan_side else "1000000")
    monkeypatch.setenv("HVAE_ENC_LAZY_READ", "1" if lazy_read else "0")
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


@pytest.mark.parametrize("graphs", [True, False])
@pytest.mark.parametrize("wd,at", [(0.0, "fwd"), (0.01, "fwd"), (0.0, "sweep")])
def test_deferred_adam_is_bitwise(hip_device, wd, at, graphs, monkeypatch):
    """The deferred W1t update (HVAE_ADAM_DEFER=1: hvae_adam_lazy_defer records a step's gradient rows, the next
    step's CSR catch-up applies it to its batch's rows and hvae_adam_lazy_pending to the rest on the defer stream)
    leaves losses, parameters and both moments bitwise those of the undeferred update: over graph-replayed (or
    eager) epochs of deferring B = 32 steps, each followed by a short 2-user tail that does not defer (the pending
    update resolved eagerly before it), an epoch at another batch size, and validation. wd != 0: the catch-up's
    full-store branch; at = sweep: the pending rows moved beside the finalize instead of the forward."""
    monkeypatch.setenv("HVAE_PLAN_SIDE_MIN_BATCH", "32")  # B = 32 defers, the tail of 2 does not
    monkeypatch.setenv("HVAE_ENC_LAZY_READ", "0")
    monkeypatch.setenv("HVAE_DEFER_AT", at)
    from hvae.executor import ConstBeta, FusedTrainer
    from src.ml.model import HybridVAE
    X = synth_csr(290, 700, seed=13)
    E = synth_embeddings(700, 128, seed=14)
    outs = []
    for defer in ("0", "1"):
        monkeypatch.setenv("HVAE_ADAM_DEFER", defer)
        torch.manual_seed(0)
        model = HybridVAE(700, E, latent_dim=64, hidden_dims=[128], dropout=0.3, beta=0.2).to(hip_device)
        fused = FusedTrainer(model, hip_device, weight_decay=wd, precision="bf16", seed=77, use_graphs=graphs)
        assert fused.adam_defer == (defer == "1") and fused._defers(32) == (defer == "1") and not fused._defers(2)
        data = fused.device_data(X, list(range(290)))
        gen = torch.Generator().manual_seed(6)
        r = [fused.run_epoch(data, 32, True, ConstBeta(0.2), 0.3, generator=gen) for _ in range(3)]
        r.append(fused.run_epoch(data, 48, True, ConstBeta(0.2), 0.3, generator=gen))
        v = fused.run_epoch(data, 32, False, ConstBeta(0.2), 0.3)
        outs.append((r, v, fused.flat.clone(), fused.m.clone(), fused.v.clone(), int(fused.step_dev.item())))
    (ra, va, fa, ma, sa, na), (rb, vb, fb, mb, sb, nb) = outs
    assert na == nb
    assert ra == rb and va == vb
    assert torch.equal(fa, fb) and torch.equal(ma, mb) and torch.equal(sa, sb)


def test_annealed_epoch_graph_is_bitwise_eager(hip_device):
    """AnnealedVAE (reference src/ml/model.py:295-334, stepped once per train batch, src/ml/train.py:74-76): the
    schedule evaluated on the device inside the captured step (AnnealedBeta -> hvae_anneal_beta) replays one graph
    per batch and gives bit for bit the epochs of the eager step fed the host's Python-float beta per batch."""
    from hvae.executor import AnnealedBeta, FusedTrainer
    from src.ml.model import create_hybrid_vae
    X = synth_csr(300, 500, seed=3)
    E = synth_embeddings(500, 128, seed=4)
    outs = []
    for arm in ("graph", "eager", "host"):
        torch.manual_seed(0)
        model = create_hybrid_vae(500, E, latent_dim=64, hidden_dims=[128], dropout=0.3, beta=0.2,
                                  use_annealing=True, anneal_steps=7).to(hip_device)
        fused = FusedTrainer(model, hip_device, precision="bf16", seed=1234, use_graphs=(arm == "graph"))
        data = fused.device_data(X, list(range(300)))
        gen = torch.Generator().manual_seed(5)
        if arm == "host":  # a plain schedule callable: eager steps, beta passed from the host per batch
            def beta_fn(_i, m=model):
                b = m.get_current_beta()
                m.step_annealing()
                return b
        else:
            beta_fn = AnnealedBeta(model)
        r = [fused.run_epoch(data, 64, True, beta_fn, 0.3, generator=gen) for _ in range(2)]
        outs.append((r, fused.flat.clone(), model.current_step))
    (ra, fa, sa), (rb, fb, sb), (rc, fc, sc) = outs
    assert sa == sb == sc == 10  # 5 batches per epoch (the last one short) x 2 epochs, past anneal_steps = 7
    assert ra == rb == rc
    assert torch.equal(fa, fb) and torch.equal(fa, fc)
