"""CPU oracle: a plain fp32 restatement of the reference HybridVAE train/eval path.

TEST INFRASTRUCTURE ONLY. Nothing in the product path (recommendation-system_amd/)
imports this module; only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it, as the checker / the timed CPU baseline.

Parity is pinned: tests/test_oracle_golden.py checks every function below
against golden vectors produced by importing the reference itself
(tests/golden/make_golden.py, committed with its outputs).

Reference = Aymane-Nouhail/Recommendation-System at /root/reference:
  model   src/ml/model.py      (HybridVAE, vae_loss_function, AnnealedVAE)
  trainer src/ml/train.py      (VAETrainer.train_epoch, _build_matrix)
  eval    src/ml/evaluate.py   (metrics, RecommendationEvaluator)
Randomness (dropout masks, reparameterisation noise) is injected explicitly,
so a train step is a pure function of its inputs.
"""
from __future__ import annotations

import math

import numpy as np
import torch

LN_EPS = 1e-5  # nn.LayerNorm default (src/ml/model.py:115)


# --------------------------------------------------------------- params ---
def init_params(n_items: int, item_embeddings: np.ndarray, latent_dim: int, hidden_dims: list[int],
                seed: int | None = None) -> dict[str, torch.Tensor]:
    """Parameters with the reference's names, shapes and RNG consumption.

    HybridVAE.__init__ (src/ml/model.py:57-101) builds nn.Linear layers in the
    order encoder..., fc_mu, fc_logvar, projection (each Linear draws its default
    reset_parameters), then _init_weights (:129-136) re-draws every Linear weight
    with kaiming_normal_(nonlinearity="relu") and zeroes the biases, in
    module-registration order. Replaying the same draws gives bit-identical
    parameters for the same torch seed.
    """
    if seed is not None:
        torch.manual_seed(seed)
    d = item_embeddings.shape[1]
    linears: list[tuple[str, torch.nn.Linear]] = []
    p: dict[str, torch.Tensor] = {"item_embeddings": torch.as_tensor(np.asarray(item_embeddings), dtype=torch.float32)}
    in_dim = n_items
    idx = 0
    for hd in hidden_dims:  # src/ml/model.py:111-120
        lin = torch.nn.Linear(in_dim, hd)
        linears.append((f"encoder.{idx}", lin))
        p[f"encoder.{idx + 1}.weight"] = torch.ones(hd)
        p[f"encoder.{idx + 1}.bias"] = torch.zeros(hd)
        idx += 4
        in_dim = hd
    linears.append(("fc_mu", torch.nn.Linear(in_dim, latent_dim)))  # :126
    linears.append(("fc_logvar", torch.nn.Linear(in_dim, latent_dim)))  # :127
    if latent_dim != d:  # :89-95
        linears.append(("projection_layer.0", torch.nn.Linear(latent_dim, d)))
        linears.append(("projection_layer.3", torch.nn.Linear(d, d)))
    for name, lin in linears:  # _init_weights, :131-136
        torch.nn.init.kaiming_normal_(lin.weight, nonlinearity="relu")
        torch.nn.init.constant_(lin.bias, 0.0)
        p[f"{name}.weight"] = lin.weight.detach().clone()
        p[f"{name}.bias"] = lin.bias.detach().clone()
    return p


def hidden_layout(p: dict[str, torch.Tensor]) -> list[int]:
    out, i = [], 0
    while f"encoder.{i}.weight" in p:
        out.append(p[f"encoder.{i}.weight"].shape[0])
        i += 4
    return out


# -------------------------------------------------------------- forward ---
def gelu(x: torch.Tensor) -> torch.Tensor:
    """nn.GELU() (exact erf form), src/ml/model.py:116, 92."""
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """nn.LayerNorm(H), biased variance, eps 1e-5 (src/ml/model.py:115)."""
    mean = x.mean(dim=-1, keepdim=True)
    var = ((x - mean) ** 2).mean(dim=-1, keepdim=True)
    return (x - mean) / torch.sqrt(var + LN_EPS) * w + b


def forward(p: dict[str, torch.Tensor], x: torch.Tensor, train: bool,
            enc_masks: list[torch.Tensor] | None = None, proj_mask: torch.Tensor | None = None,
            eps: torch.Tensor | None = None) -> dict[str, torch.Tensor]:
    """HybridVAE.forward (src/ml/model.py:202-221) with explicit randomness.

    enc_masks[k] / proj_mask are the Dropout multipliers (0 or 1/(1-p)); eps
    replaces torch.randn_like in reparameterize (:173). In eval mode dropout is
    the identity and z = mu (:168-179).
    """
    h = x
    for k, _ in enumerate(hidden_layout(p)):  # encode, :149 (Sequential of :112-118)
        i = 4 * k
        h = h @ p[f"encoder.{i}.weight"].t() + p[f"encoder.{i}.bias"]
        h = gelu(layer_norm(h, p[f"encoder.{i + 1}.weight"], p[f"encoder.{i + 1}.bias"]))
        if train and enc_masks is not None:
            h = h * enc_masks[k]
    mu = h @ p["fc_mu.weight"].t() + p["fc_mu.bias"]  # :152
    logvar = h @ p["fc_logvar.weight"].t() + p["fc_logvar.bias"]  # :153
    if train:  # reparameterize, :168-176
        std = torch.exp(0.5 * logvar)
        z = mu + eps * std
    else:
        z = mu
    if "projection_layer.0.weight" in p:  # decode, :195 (Sequential of :90-95)
        a = z @ p["projection_layer.0.weight"].t() + p["projection_layer.0.bias"]
        g = gelu(a)
        if train and proj_mask is not None:
            g = g * proj_mask
        u = g @ p["projection_layer.3.weight"].t() + p["projection_layer.3.bias"]
    else:
        u = z
    scores = u @ p["item_embeddings"].t()  # :198
    return {"scores": scores, "mu": mu, "logvar": logvar, "z": z, "u": u}


def vae_loss(scores: torch.Tensor, x: torch.Tensor, mu: torch.Tensor, logvar: torch.Tensor,
             beta: float) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """vae_loss_function (src/ml/model.py:259-292)."""
    lse = torch.logsumexp(scores, dim=-1, keepdim=True)
    recon = -torch.mean(torch.sum(x * (scores - lse), dim=-1))  # :281
    kl = -0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp()) / x.shape[0]  # :286-287
    return recon + beta * kl, recon, kl  # :290


# ---------------------------------------------------------- train step ---
PARAM_ORDER_NOTE = "reference model.parameters() order: encoder..., fc_mu, fc_logvar, projection_layer"


def param_names(p: dict[str, torch.Tensor]) -> list[str]:
    """Trainable parameters in the reference's model.parameters() order (E is a buffer)."""
    names = []
    for k, _ in enumerate(hidden_layout(p)):
        i = 4 * k
        names += [f"encoder.{i}.weight", f"encoder.{i}.bias", f"encoder.{i + 1}.weight", f"encoder.{i + 1}.bias"]
    names += ["fc_mu.weight", "fc_mu.bias", "fc_logvar.weight", "fc_logvar.bias"]
    if "projection_layer.0.weight" in p:
        names += ["projection_layer.0.weight", "projection_layer.0.bias",
                  "projection_layer.3.weight", "projection_layer.3.bias"]
    return names


def grads(p: dict[str, torch.Tensor], x: torch.Tensor, beta: float, enc_masks=None, proj_mask=None, eps=None,
          train_e: bool = False):
    """loss.backward() of VAETrainer.train_epoch (src/ml/train.py:88-90) -> (grads, losses). train_e: E is a
    parameter too (HybridVAE(freeze_embeddings=False), src/ml/model.py:72-75; the first in parameters() order)."""
    names = (["item_embeddings"] if train_e else []) + param_names(p)
    q = {k: (v.detach().clone().requires_grad_(k in names)) for k, v in p.items()}
    out = forward(q, x, True, enc_masks, proj_mask, eps)
    loss, recon, kl = vae_loss(out["scores"], x, out["mu"], out["logvar"], beta)
    g = torch.autograd.grad(loss, [q[n] for n in names])
    return {n: gi.detach() for n, gi in zip(names, g)}, (loss.item(), recon.item(), kl.item())


def clip_coef(g: dict[str, torch.Tensor], max_norm: float = 5.0) -> tuple[float, float]:
    """clip_grad_norm_(params, 5.0) (src/ml/train.py:91): norm of per-tensor norms."""
    norms = torch.stack([torch.linalg.vector_norm(t, 2.0) for t in g.values()])
    total = torch.linalg.vector_norm(norms, 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    return float(total), float(coef)


def adam_update(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int, lr: float = 1e-3,
                betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
    """torch.optim.Adam single-tensor step (src/ml/train.py:63, 92), in place."""
    if weight_decay != 0:
        g = g + weight_decay * p
    m.lerp_(g, 1 - betas[0])
    v.mul_(betas[1]).addcmul_(g, g, value=1 - betas[1])
    bc1 = 1 - betas[0] ** step
    bc2 = 1 - betas[1] ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-(lr / bc1))


def train_step(p: dict[str, torch.Tensor], state: dict, x: torch.Tensor, beta: float, lr: float = 1e-3,
               weight_decay: float = 0.0, enc_masks=None, proj_mask=None, eps=None, train_e: bool = False) -> dict:
    """One VAETrainer.train_epoch batch (src/ml/train.py:86-96): fwd, bwd, clip 5.0, Adam (train_e: on E too)."""
    g, losses = grads(p, x, beta, enc_masks, proj_mask, eps, train_e)
    total, coef = clip_coef(g)
    state["step"] = state.get("step", 0) + 1
    for n, gi in g.items():
        if n not in state:
            state[n] = (torch.zeros_like(p[n]), torch.zeros_like(p[n]))
        m, v = state[n]
        adam_update(p[n], gi * coef, m, v, state["step"], lr=lr, weight_decay=weight_decay)
    return {"grads": g, "loss": losses, "total_norm": total, "coef": coef}


class CpuTrainer:
    """The reference's train step as its own modules run it, for bench.py's cpu_baseline leg.

    train_step above is the checker (explicit tensors, autograd.grad on clones); this class is the same
    math laid out the way VAETrainer.train_epoch executes it (src/ml/train.py:81-103), so that its CPU
    time stands for the reference's: nn.Linear / nn.LayerNorm / nn.GELU / nn.Dropout in the encoder's
    Sequential order (src/ml/model.py:103-136), F.log_softmax in the loss (:259-292), loss.backward(),
    clip_grad_norm_(5.0) and torch.optim.Adam over model.parameters() order. Dropout masks and the
    reparameterisation noise may be injected (then the step equals train_step's;
    tests/test_oracle_golden.py pins that), else they are drawn as the reference draws them.
    """

    def __init__(self, p: dict[str, torch.Tensor], dropout: float, lr: float = 1e-3, weight_decay: float = 0.0):
        nn = torch.nn
        self.dropout = dropout
        enc = []
        for k, h in enumerate(hidden_layout(p)):
            i = 4 * k
            lin = nn.Linear(p[f"encoder.{i}.weight"].shape[1], h)
            ln = nn.LayerNorm(h)
            with torch.no_grad():
                lin.weight.copy_(p[f"encoder.{i}.weight"]); lin.bias.copy_(p[f"encoder.{i}.bias"])
                ln.weight.copy_(p[f"encoder.{i + 1}.weight"]); ln.bias.copy_(p[f"encoder.{i + 1}.bias"])
            enc.append((lin, ln))
        self.enc = enc

        def linear(name):
            w = p[f"{name}.weight"]
            m = nn.Linear(w.shape[1], w.shape[0])
            with torch.no_grad():
                m.weight.copy_(w); m.bias.copy_(p[f"{name}.bias"])
            return m
        self.fc_mu, self.fc_logvar = linear("fc_mu"), linear("fc_logvar")
        self.proj = (linear("projection_layer.0"), linear("projection_layer.3")) \
            if "projection_layer.0.weight" in p else None
        self.E = p["item_embeddings"]
        params = []
        for lin, ln in enc:
            params += [lin.weight, lin.bias, ln.weight, ln.bias]
        params += [self.fc_mu.weight, self.fc_mu.bias, self.fc_logvar.weight, self.fc_logvar.bias]
        if self.proj:
            params += [self.proj[0].weight, self.proj[0].bias, self.proj[1].weight, self.proj[1].bias]
        self.params = params
        self.opt = torch.optim.Adam(params, lr=lr, weight_decay=weight_decay)

    def _drop(self, h, mask):
        return h * mask if mask is not None else torch.nn.functional.dropout(h, self.dropout, training=True)

    def step(self, x: torch.Tensor, beta: float, enc_masks=None, proj_mask=None, eps=None) -> float:
        F = torch.nn.functional
        self.opt.zero_grad()
        h = x
        for k, (lin, ln) in enumerate(self.enc):
            h = self._drop(F.gelu(ln(lin(h))), enc_masks[k] if enc_masks is not None else None)
        mu, logvar = self.fc_mu(h), self.fc_logvar(h)
        std = torch.exp(0.5 * logvar)
        z = mu + (eps if eps is not None else torch.randn_like(std)) * std
        u = z
        if self.proj:
            u = self.proj[1](self._drop(F.gelu(self.proj[0](z)), proj_mask))
        scores = u @ self.E.t()
        recon = -torch.mean(torch.sum(x * F.log_softmax(scores, dim=-1), dim=-1))
        kl = -0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp()) / x.shape[0]
        loss = recon + beta * kl
        loss.backward()
        torch.nn.utils.clip_grad_norm_(self.params, max_norm=5.0)
        self.opt.step()
        return float(loss.item())

    def state(self) -> dict[str, torch.Tensor]:
        """Parameters under the reference's state-dict names (for the pinning test)."""
        out = {}
        for k, (lin, ln) in enumerate(self.enc):
            i = 4 * k
            out[f"encoder.{i}.weight"], out[f"encoder.{i}.bias"] = lin.weight, lin.bias
            out[f"encoder.{i + 1}.weight"], out[f"encoder.{i + 1}.bias"] = ln.weight, ln.bias
        out["fc_mu.weight"], out["fc_mu.bias"] = self.fc_mu.weight, self.fc_mu.bias
        out["fc_logvar.weight"], out["fc_logvar.bias"] = self.fc_logvar.weight, self.fc_logvar.bias
        if self.proj:
            out["projection_layer.0.weight"], out["projection_layer.0.bias"] = self.proj[0].weight, self.proj[0].bias
            out["projection_layer.3.weight"], out["projection_layer.3.bias"] = self.proj[1].weight, self.proj[1].bias
        return {k: v.detach() for k, v in out.items()}


# ------------------------------------------------------------------ data ---
def build_matrix(users: np.ndarray, items: np.ndarray, binary: np.ndarray | None, shape) -> "scipy.sparse.csr_matrix":
    """_build_matrix (src/ml/train.py:175-182): positives only, duplicates summed."""
    from scipy.sparse import csr_matrix
    keep = np.ones(len(users), bool) if binary is None else (np.asarray(binary) == 1)
    return csr_matrix((np.ones(int(keep.sum())), (np.asarray(users)[keep], np.asarray(items)[keep])), shape=shape)


# --------------------------------------------------------------- metrics ---
def recall_at_k(recommended, relevant, k):  # src/ml/evaluate.py:32-37
    if len(relevant) == 0:
        return 0.0
    return len(np.intersect1d(np.asarray(recommended)[:k], relevant)) / len(relevant)


def ndcg_at_k(recommended, relevant, k):  # src/ml/evaluate.py:40-47
    if len(relevant) == 0:
        return 0.0
    rel = set(np.asarray(relevant).tolist())
    dcg = sum(1.0 / np.log2(i + 2) for i, item in enumerate(np.asarray(recommended)[:k]) if item in rel)
    idcg = sum(1.0 / np.log2(i + 2) for i in range(min(len(relevant), k)))
    return dcg / idcg if idcg > 0 else 0.0


def hit_ratio_at_k(recommended, relevant, k):  # src/ml/evaluate.py:50-54
    if len(relevant) == 0:
        return 0.0
    return 1.0 if len(np.intersect1d(np.asarray(recommended)[:k], relevant)) > 0 else 0.0


def rank_candidates(scores_row: np.ndarray, candidates: np.ndarray) -> np.ndarray:
    """candidates[np.argsort(scores[candidates])[::-1]] (src/ml/evaluate.py:173-175),
    with a stable argsort so that ties have one defined order."""
    return candidates[np.argsort(scores_row[candidates], kind="stable")[::-1]]


def topk_exclude_seen(scores_row: np.ndarray, seen: np.ndarray, k: int) -> np.ndarray:
    """get_user_recommendations (src/ml/evaluate.py:137-147), stable argsort."""
    s = scores_row.astype(np.float32).copy()
    s[seen] = -np.inf
    return np.argsort(s, kind="stable")[::-1][:k]
