"""Trainable item embeddings (HybridVAE(freeze_embeddings=False), reference src/ml/model.py:72-75): E is a
parameter, VAETrainer trains it with the rest (reference src/ml/train.py:81-103: fwd, loss, backward,
clip_grad_norm_(5.0), Adam). On MI355X this runs the module-API step on libhvae kernels (scores materialised per
batch, as in the reference) with ModuleAdam (hvae_adam_dense + hvae_clip_grad_norm).

Checked against the oracle (oracle/ref_cpu.py, pinned to the reference's golden vectors): the gradients of every
parameter including E in eval mode (deterministic: z = mu, dropout off), one clipped Adam step on them, and a
training epoch through VAETrainer."""
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
    assert trainer.fused is None
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
