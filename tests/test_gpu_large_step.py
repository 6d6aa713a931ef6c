"""The whole fused train step against the oracle at the BASELINE shapes.

configs[2] Syn-1M (4096 users x 100,000 items, d = 384) and configs[3] the Syn-10M shard (4096 x 1,000,000,
d = 768), bf16 decoder at both, and configs[4] (fp8 decoder) at the Syn-10M shard; latent 128, hidden [512]
(SURVEY §8). Dropout masks and the reparameterisation noise are injected, so a step is a pure function of its
inputs. The oracle (oracle/ref_cpu.train_step: the reference's forward, vae_loss_function, loss.backward(),
clip_grad_norm_(5.0) and torch.optim.Adam, src/ml/model.py:138-221, 259-292, src/ml/train.py:86-96) runs in
fp32 on the same device with a dense x (B x N: 1.6 GB / 16 GB) -- the reference's own dense formulation,
which fits 288 GB of HBM many times over.

Two steps from the same init (HybridVAE and the oracle draw identical parameters, tests/test_api_cpu.py):
the losses and clip norm of both steps, every pre-clip gradient of step 1 (the first layer's from its
row-sparse form), and parameters, Adam m and v after step 2, at the bars of
tests/test_gpu_train.py::STEP_TOL -- the same bars as the small golden shapes.

The three checks in one pass cover what the per-kernel large-shape tests do not: the CSR catch-up of lazy
Adam, the row-gradient plan on its own stream, the split-K weight-gradient GEMMs and the chunk-cut row-gradient
apply, all at B = 4096.
"""
import numpy as np
import pytest
import torch

from gen import synth_csr, synth_embeddings
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu

CASES = {
    "syn1m_bf16": dict(B=4096, N=100_000, d=384, precision="bf16", seed=61),
    "syn10m_bf16": dict(B=4096, N=1_000_000, d=768, precision="bf16", seed=62),
    "syn10m_fp8": dict(B=4096, N=1_000_000, d=768, precision="fp8", seed=63),
}
L, H, P_DROP, BETA, LR = 128, [512], 0.3, 0.2, 1e-3


def _maxrel(a, b):
    a = a.detach().double()
    b = b.detach().double().to(a.device)
    return float((a - b).abs().max() / max(b.abs().max().item(), 1e-30))


def _rms_lr(a, b):
    d = a.detach().double() - b.detach().double().to(a.device)
    return float(d.pow(2).mean().sqrt()) / LR


@pytest.mark.timeout(900)
@pytest.mark.parametrize("case", sorted(CASES))
def test_fused_step_vs_oracle_full_shape(hip_device, case):
    from test_gpu_train import STEP_TOL

    from hvae import ops
    from hvae.executor import FusedTrainer
    from src.ml.model import HybridVAE
    c = CASES[case]
    B, N, d, dev = c["B"], c["N"], c["d"], hip_device
    X = synth_csr(B, N, lam=15.0, seed=c["seed"])
    E = synth_embeddings(N, d, seed=c["seed"] + 1)
    g = torch.Generator(device=dev).manual_seed(c["seed"] + 2)

    def ext():
        return {"enc_masks": [(torch.rand(B, H[0], device=dev, generator=g) >= P_DROP).float() / (1 - P_DROP)],
                "proj_mask": (torch.rand(B, d, device=dev, generator=g) >= P_DROP).float() / (1 - P_DROP),
                "eps": torch.randn(B, L, device=dev, generator=g)}
    steps = [ext(), ext()]

    # ---- the fused MI355X step (graph-free: step_batch is the eager form of the captured step)
    torch.manual_seed(c["seed"])
    model = HybridVAE(N, E, latent_dim=L, hidden_dims=H, dropout=P_DROP, beta=BETA).to(dev)
    fused = FusedTrainer(model, dev, lr=LR, precision=c["precision"], use_graphs=False)
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
    got_p = {n: p.detach().clone() for n, p in model.named_parameters()}
    got_m = {n: (fused.m_w1t.t() if n == "encoder.0.weight" else lay.view(fused.m, n)).clone() for n in got_p}
    got_v = {n: (fused.v_w1t.t() if n == "encoder.0.weight" else lay.view(fused.v, n)).clone() for n in got_p}
    del fused, model, data
    torch.cuda.empty_cache()

    # ---- the oracle: the reference's dense fp32 step on the same device
    p = {k: v.to(dev) for k, v in R.init_params(N, E, L, H, seed=c["seed"]).items()}
    x = torch.zeros(B, N, device=dev)
    xc = ops.csr_from_scipy(X, dev)
    rows = torch.repeat_interleave(torch.arange(B, device=dev), xc.row_ptr[1:] - xc.row_ptr[:-1])
    x.index_put_((rows, xc.col_idx.long()), xc.vals, accumulate=True)
    state, ref = {}, []
    for s in range(2):
        ref.append(R.train_step(p, state, x, BETA, lr=LR, enc_masks=steps[s]["enc_masks"],
                                proj_mask=steps[s]["proj_mask"], eps=steps[s]["eps"]))
        if s == 0:
            ref_grad = {n: t.clone() for n, t in ref[0]["grads"].items()}
        ref[-1]["grads"] = None
    del x
    torch.cuda.synchronize()

    tol = STEP_TOL[c["precision"]]
    err = {}
    for s in range(2):
        want = np.asarray(ref[s]["loss"])
        err[f"loss:{s}"] = float(np.max(np.abs(got_loss[s] - want) / np.abs(want)))
        err[f"norm:{s}"] = abs(got_norm[s] - ref[s]["total_norm"]) / ref[s]["total_norm"]
    for n, t in ref_grad.items():
        err[f"grad:{n}"] = _maxrel(got_grad[n], t)
    for n, t in got_p.items():
        m, v = state[n]
        err[f"param:{n}"] = _rms_lr(t, p[n])
        err[f"m:{n}"] = _maxrel(got_m[n], m)
        err[f"v:{n}"] = _maxrel(got_v[n], v)
    print(case, {k: f"{e:.2e}" for k, e in err.items()})
    bad = {k: e for k, e in err.items() if not e <= tol[k.split(":")[0]]}
    assert not bad, (case, bad)
