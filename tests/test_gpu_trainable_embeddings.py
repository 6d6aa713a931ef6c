"""Trainable item embeddings (HybridVAE(freeze_embeddings=False), reference src/ml/model.py:72-75): E is a
parameter, VAETrainer trains it with the rest (reference src/ml/train.py:81-103: fwd, loss, backward,
clip_grad_norm_(5.0), Adam). On MI355X this runs the module-API step on libhvae kernels (scores materialised per
batch, as in the reference) with ModuleAdam (hvae_adam_dense + hvae_clip_grad_norm).

Checked against the oracle (oracle/ref_cpu.py, pinned to the reference's golden vectors): the gradients of every
parameter including E in eval mode (deterministic: z = mu, dropout off), one clipped Adam step on them, and a
training epoch through VAETrainer.

Round 6: VAETrainer runs trainable E on the fused step (hvae/executor.py: E in the flat dense segment, its
decoder image refreshed each step, dE's dense term in item chunks and its sparse term through the W1 row-gradient
plan, hvae_embed.hip); two such steps with injected dropout masks and noise match the oracle's train_step(train_e)
at tests/test_gpu_train.py::STEP_TOL, at a small shape (fp32, bf16) and at the Syn-1M shape (bf16, B = 4096,
100,000 items, d = 384). The module-API step stays for HVAE_TRAINABLE_E_MODULE=1."""
import numpy as np
import pytest
import torch

from gen import synth_csr, synth_embeddings
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu


def _maxrel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-30))


def _setup(hip_device, n_users=24, n_items=300, d=128, latent=64, hidden=(128,), seed=5):
    from src.ml.model import HybridVAE
    X = synth_csr(n_users, n_items, lam=4.0, seed=seed)
    E = synth_embeddings(n_items, d, seed=seed + 1)
    torch.manual_seed(seed)
    model = HybridVAE(n_items, E, latent_dim=latent, hidden_dims=list(hidden), dropout=0.3, beta=0.2,
                      freeze_embeddings=False).to(hip_device)
    p = R.init_params(n_items, E, latent, list(hidden), seed=seed)
    return X, E, model, p


def _oracle_grads(p, x, beta):
    names = R.param_names(p) + ["item_embeddings"]
    q = {k: v.detach().clone().requires_grad_(k in names) for k, v in p.items()}
    out = R.forward(q, x, False)
    loss, _, _ = R.vae_loss(out["scores"], x, out["mu"], out["logvar"], beta)
    g = torch.autograd.grad(loss, [q[n] for n in names])
    return dict(zip(names, g)), loss.item()


def test_trainable_E_gradients_and_adam_step(hip_device):
    from src.ml.model import vae_loss_function
    from src.ml.train import ModuleAdam
    X, E, model, p = _setup(hip_device)
    x = torch.as_tensor(X.toarray(), dtype=torch.float32)
    assert isinstance(model.item_embeddings, torch.nn.Parameter)
    # eval-mode gradients (z = mu, no dropout): every parameter, E included
    model.eval()
    recon_x, mu, logvar = model(x.to(hip_device))
    loss, _, _ = vae_loss_function(recon_x, x.to(hip_device), mu, logvar, 0.2)
    loss.backward()
    g_ref, loss_ref = _oracle_grads(p, x, 0.2)
    assert abs(loss.item() - loss_ref) < 1e-5 * abs(loss_ref)
    named = dict(model.named_parameters())
    for n, gr in g_ref.items():
        assert _maxrel(named[n].grad, gr) < 1e-4, n
    # one clipped Adam step (clip_grad_norm_ 5.0 + torch Adam), E included
    opt = ModuleAdam(model.parameters(), lr=1e-3)
    opt.step(max_norm=5.0)
    total, coef = R.clip_coef(g_ref)
    assert abs(opt.norm.item() - total) < 1e-4 * total
    for n, gr in g_ref.items():
        ref = p[n].clone()
        R.adam_update(ref, gr * coef, torch.zeros_like(ref), torch.zeros_like(ref), 1)
        # Adam's first step is ~lr * sign(g): in units of lr, exact where the gradient is clearly nonzero (a
        # near-zero gradient's sign is rounding noise and may flip, moving its element by 2 lr)
        dev = (named[n].detach().cpu().double() - ref.double()).abs() / 1e-3
        big = gr.abs() > 1e-3 * gr.abs().max()
        assert float(dev[big].max()) < 1e-2, n
        assert float(dev.pow(2).mean().sqrt()) < 0.05, n
    sd = opt.state_dict()
    assert int(sd["state"][0]["step"]) == 1 and len(sd["state"]) == len(named)


def test_trainer_trains_embeddings(hip_device, tmp_path):
    from src.ml.train import UserInteractionDataset, VAETrainer
    X, E, model, p = _setup(hip_device, n_users=96)
    E0 = model.item_embeddings.detach().clone()
    trainer = VAETrainer(model, hip_device, lr=1e-3)
    assert trainer.fused is not None and trainer.fused.train_e  # the fused step, E in its dense segment
    loader = torch.utils.data.DataLoader(UserInteractionDataset(X), batch_size=16, shuffle=True)
    m1 = trainer.train_epoch(loader)
    m2 = trainer.train_epoch(loader)
    v = trainer.validate(torch.utils.data.DataLoader(UserInteractionDataset(X), batch_size=16))
    assert m2["total_loss"] < m1["total_loss"] and np.isfinite(v["total_loss"])
    assert not torch.equal(model.item_embeddings.detach(), E0)  # E moved
    trainer.save_checkpoint(tmp_path / "c.pth", 2)
    ck = torch.load(tmp_path / "c.pth", map_location=hip_device, weights_only=True)
    assert "item_embeddings" in ck["model_state_dict"]
    assert torch.equal(ck["model_state_dict"]["item_embeddings"], model.item_embeddings.detach())


def test_trainer_trains_embeddings_module_path(hip_device, monkeypatch):
    from src.ml.train import UserInteractionDataset, VAETrainer
    monkeypatch.setenv("HVAE_TRAINABLE_E_MODULE", "1")
    X, E, model, p = _setup(hip_device, n_users=64)
    E0 = model.item_embeddings.detach().clone()
    trainer = VAETrainer(model, hip_device, lr=1e-3)
    assert trainer.fused is None
    loader = torch.utils.data.DataLoader(UserInteractionDataset(X), batch_size=16, shuffle=True)
    m1 = trainer.train_epoch(loader)
    assert np.isfinite(m1["total_loss"]) and not torch.equal(model.item_embeddings.detach(), E0)


def _fused_vs_oracle(hip_device, B, N, d, L, H, precision, seed):
    """Two fused steps with trainable E (injected masks and noise) against the oracle's train_step(train_e=True)."""
    from test_gpu_train import STEP_TOL

    from hvae import ops
    from hvae.executor import FusedTrainer
    from src.ml.model import HybridVAE
    P_DROP, BETA, LR = 0.3, 0.2, 1e-3
    dev = hip_device
    X = synth_csr(B, N, lam=15.0 if B >= 1024 else 5.0, seed=seed)
    E = synth_embeddings(N, d, seed=seed + 1)
    g = torch.Generator(device=dev).manual_seed(seed + 2)

    def ext():
        return {"enc_masks": [(torch.rand(B, H[0], device=dev, generator=g) >= P_DROP).float() / (1 - P_DROP)],
                "proj_mask": (torch.rand(B, d, device=dev, generator=g) >= P_DROP).float() / (1 - P_DROP),
                "eps": torch.randn(B, L, device=dev, generator=g)}
    steps = [ext(), ext()]
    torch.manual_seed(seed)
    model = HybridVAE(N, E, latent_dim=L, hidden_dims=H, dropout=P_DROP, beta=BETA, freeze_embeddings=False).to(dev)
    fused = FusedTrainer(model, dev, lr=LR, precision=precision, use_graphs=False)
    assert fused.train_e
    data = fused.device_data(X, list(range(B)))
    got_loss, got_norm = [], []
    for s in range(2):
        got_loss.append(fused.step_batch(data, None, B, BETA, P_DROP, train=True, ext=steps[s]).cpu().numpy())
        got_norm.append(fused.norm.item())
        if s == 0:
            bf = fused._bufs[(B, True)]
            w1 = torch.zeros(N, H[0], device=dev)
            ops.rowgrad_to_dense(bf.rg, w1)
            gW, gb = fused.gW_heads, fused.gb_heads
            got_grad = {"encoder.0.weight": w1.t().contiguous(), "fc_mu.weight": gW[:L].clone(),
                        "fc_logvar.weight": gW[L:].clone(), "fc_mu.bias": gb[:L].clone(),
                        "fc_logvar.bias": gb[L:].clone()}
            for n, t in fused.G.items():
                got_grad[n] = t.clone()
            del w1
    torch.cuda.synchronize()
    lay = fused.layout
    got_p = {n: q.detach().clone() for n, q in model.named_parameters()}
    assert "item_embeddings" in got_p
    got_m = {n: (fused.m_w1t.t() if n == "encoder.0.weight" else lay.view(fused.m, n)).clone() for n in got_p}
    got_v = {n: (fused.v_w1t.t() if n == "encoder.0.weight" else lay.view(fused.v, n)).clone() for n in got_p}
    del fused, model, data
    torch.cuda.empty_cache()
    p = {k: v.to(dev) for k, v in R.init_params(N, E, L, H, seed=seed).items()}
    x = torch.zeros(B, N, device=dev)
    xc = ops.csr_from_scipy(X, dev)
    rows = torch.repeat_interleave(torch.arange(B, device=dev), xc.row_ptr[1:] - xc.row_ptr[:-1])
    x.index_put_((rows, xc.col_idx.long()), xc.vals, accumulate=True)
    state, ref = {}, []
    for s in range(2):
        ref.append(R.train_step(p, state, x, BETA, lr=LR, enc_masks=steps[s]["enc_masks"],
                                proj_mask=steps[s]["proj_mask"], eps=steps[s]["eps"], train_e=True))
        if s == 0:
            ref_grad = {n: t.clone() for n, t in ref[0]["grads"].items()}
        ref[-1]["grads"] = None
    del x
    torch.cuda.synchronize()
    assert "item_embeddings" in ref_grad and "item_embeddings" in state
    tol = STEP_TOL[precision]
    err = {}
    for s in range(2):
        want = np.asarray(ref[s]["loss"])
        err[f"loss:{s}"] = float(np.max(np.abs(got_loss[s] - want) / np.abs(want)))
        err[f"norm:{s}"] = abs(got_norm[s] - ref[s]["total_norm"]) / ref[s]["total_norm"]
    for n, t in ref_grad.items():
        err[f"grad:{n}"] = _maxrel(got_grad[n], t)
    for n, t in got_p.items():
        m, v = state[n]
        err[f"param:{n}"] = float((t.double() - p[n].double()).pow(2).mean().sqrt()) / LR
        err[f"m:{n}"] = _maxrel(got_m[n], m)
        err[f"v:{n}"] = _maxrel(got_v[n], v)
    print({k: f"{e:.2e}" for k, e in err.items() if "item_embeddings" in k or ":" in k and k[:4] in ("loss", "norm")})
    bad = {k: e for k, e in err.items() if not e <= tol[k.split(":")[0]]}
    assert not bad, bad


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_fused_trainable_E_step_small(hip_device, precision):
    _fused_vs_oracle(hip_device, B=48, N=700, d=128, L=64, H=[128], precision=precision, seed=71)


@pytest.mark.timeout(900)
def test_fused_trainable_E_step_syn1m(hip_device):
    """The Syn-1M shape (BASELINE configs[2]: B = 4096, 100,000 items, d = 384, latent 128, hidden [512]), bf16."""
    _fused_vs_oracle(hip_device, B=4096, N=100_000, d=384, L=128, H=[512], precision="bf16", seed=73)
