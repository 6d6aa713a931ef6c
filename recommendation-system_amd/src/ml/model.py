"""HybridVAE on MI355X -- drop-in for the reference's src/ml/model.py.

Same class names, constructor signatures, attributes, submodule / state_dict
layout and initialisation (RNG draws included) as the reference
(src/ml/model.py:27-385), so checkpoints load in both directions. Every
computation runs on libhvae HIP kernels (hvae/autograd.py); there is no CPU
fallback: calling the model on CPU tensors raises.

Storage difference (invisible through the API): encoder.0.weight, the
[H, N_items] first-layer weight, is kept item-major -- the Parameter is the
transposed view of a contiguous [N_items, H] tensor -- so the sparse encoder
gathers whole 2 KB item rows.
"""
from __future__ import annotations

import logging
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from hvae import ops
from hvae.autograd import EncoderFirstFn, LinearFn, LnGeluDropFn, ReparamFn, ScoresFn, VaeLossFn

logger = logging.getLogger(__name__)


class HipLinear(nn.Linear):
    """nn.Linear parameters (same init draws); forward on the fp32 MFMA GEMM."""

    def forward(self, x):
        return LinearFn.apply(x, self.weight, self.bias, False, 0.0, False)


class _FusedOnly:
    def forward(self, *_a, **_k):
        raise NotImplementedError(
            f"{type(self).__name__} is fused into its parent (LayerNorm+GELU+Dropout run as one HIP kernel); "
            "call the parent Sequential / the model instead")


class HipLayerNorm(_FusedOnly, nn.LayerNorm):
    pass


class HipGELU(_FusedOnly, nn.GELU):
    pass


class HipDropout(_FusedOnly, nn.Dropout):
    pass


class HipEncoder(nn.Sequential):
    """[Linear, LayerNorm, GELU, Dropout] * len(hidden) with the reference's indices (model.py:103-123)."""

    def forward(self, x):
        n_layers = len(self) // 4
        csr = x if isinstance(x, ops.Csr) else ops.dense_to_csr(x)
        lin0, ln0, drop0 = self[0], self[1], self[3]
        h = EncoderFirstFn.apply(lin0.weight, lin0.bias, ln0.weight, ln0.bias, csr, float(drop0.p), self.training)
        for k in range(1, n_layers):
            lin, ln, drop = self[4 * k], self[4 * k + 1], self[4 * k + 3]
            a = LinearFn.apply(h, lin.weight, lin.bias, False, 0.0, False)
            h = LnGeluDropFn.apply(a, ln.weight, ln.bias, float(drop.p), self.training, k)
        return h


class HipProjection(nn.Sequential):
    """Linear(L, d) -> GELU -> Dropout -> Linear(d, d) (model.py:89-95), first three fused."""

    def forward(self, z):
        a, drop, b = self[0], self[2], self[3]
        q = LinearFn.apply(z, a.weight, a.bias, True, float(drop.p), self.training)
        return LinearFn.apply(q, b.weight, b.bias, False, 0.0, False)


class HybridVAE(nn.Module):
    """Hybrid VAE for recommendation (reference: src/ml/model.py:27-256)."""

    def __init__(
        self,
        n_items: int,
        item_embeddings: np.ndarray,
        latent_dim: int = 200,
        hidden_dims: Optional[list] = None,
        dropout: float = 0.5,
        beta: float = 0.2,
        freeze_embeddings: bool = True,
    ):
        super().__init__()
        self.n_items = n_items
        self.latent_dim = latent_dim
        self.dropout = dropout
        self.beta = beta
        if hidden_dims is None:
            hidden_dims = [600, 200]
        self.hidden_dims = hidden_dims
        self.embedding_dim = item_embeddings.shape[1]
        self.item_embeddings_trainable = not freeze_embeddings
        if freeze_embeddings:
            self.register_buffer("item_embeddings", torch.FloatTensor(np.asarray(item_embeddings)))
        else:
            self.item_embeddings = nn.Parameter(torch.FloatTensor(np.asarray(item_embeddings)))
        logger.info("Initializing HybridVAE (MI355X): items=%d latent=%d emb=%d hidden=%s beta=%s frozen=%s",
                    n_items, latent_dim, self.embedding_dim, hidden_dims, beta, freeze_embeddings)
        self._build_encoder()
        if self.latent_dim != self.embedding_dim:
            self.projection_layer = HipProjection(
                HipLinear(self.latent_dim, self.embedding_dim),
                HipGELU(),
                HipDropout(self.dropout),
                HipLinear(self.embedding_dim, self.embedding_dim),
            )
        else:
            self.projection_layer = nn.Identity()
        self._init_weights()
        # keep the first-layer weight item-major ([N, H] storage, [H, N] view)
        w = self.encoder[0].weight
        self.encoder[0].weight = nn.Parameter(w.detach().t().contiguous().t())

    def _build_encoder(self):
        layers = []
        in_dim = self.n_items
        for hidden_dim in self.hidden_dims:
            layers.extend([HipLinear(in_dim, hidden_dim), HipLayerNorm(hidden_dim), HipGELU(),
                           HipDropout(self.dropout)])
            in_dim = hidden_dim
        self.encoder = HipEncoder(*layers)
        self.fc_mu = HipLinear(in_dim, self.latent_dim)
        self.fc_logvar = HipLinear(in_dim, self.latent_dim)

    def _init_weights(self):
        """He (kaiming_normal_, relu gain) weights, zero biases (model.py:129-136)."""
        for module in self.modules():
            if isinstance(module, nn.Linear):
                nn.init.kaiming_normal_(module.weight, nonlinearity="relu")
                if module.bias is not None:
                    nn.init.constant_(module.bias, 0.0)

    # ------------------------------------------------------------- API ---
    def encode(self, x) -> Tuple[torch.Tensor, torch.Tensor]:
        """x: dense [B, N] user rows (any values) or an hvae.ops.Csr batch."""
        if not isinstance(x, ops.Csr):
            ops.require_hip(x)
        h = self.encoder(x)
        return self.fc_mu(h), self.fc_logvar(h)

    def reparameterize(self, mu: torch.Tensor, logvar: torch.Tensor) -> torch.Tensor:
        if self.training:
            return ReparamFn.apply(mu, logvar)
        return mu

    def decode(self, z: torch.Tensor) -> torch.Tensor:
        ops.require_hip(z)
        user_embedding = self.projection_layer(z)
        return ScoresFn.apply(user_embedding, self.item_embeddings)

    def forward(self, x) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        mu, logvar = self.encode(x)
        z = self.reparameterize(mu, logvar)
        return self.decode(z), mu, logvar

    def get_user_embedding(self, x) -> torch.Tensor:
        mu, _ = self.encode(x)
        return mu

    def recommend(self, user_embedding: torch.Tensor, top_k: int = 10) -> Tuple[torch.Tensor, torch.Tensor]:
        """Exact top-k over all items (ties: larger item index first) -- reference model.py:236-256's
        torch.topk(decode(z)). The [B, N] scores are never formed: the fused bf16-shortlist / fp32-rescore
        top-K (hvae_topk_fused) ranks u = projection(z) against E."""
        with torch.no_grad():
            squeeze = user_embedding.dim() == 1
            z = user_embedding.reshape(-1, user_embedding.shape[-1])
            u = self.projection_layer(z).contiguous()
            idx, val = self.topk_scores(u, top_k)
            idx = idx.long()
            if squeeze:
                idx, val = idx[0], val[0]
        return idx, val

    def topk_scores(self, u: torch.Tensor, k: int, exclude: "ops.Csr | None" = None):
        """Exact top-k of u E^T per row (exclude: CSR rows of items left out), fused where hvae_topk_fused covers
        the shape (k <= 256, d in 64..768), else through the fp32 score matrix + hvae_topk (both on the GPU)."""
        E = self.item_embeddings.detach()
        d = E.shape[1]
        if k <= 256 and d in (64, 128, 256, 384, 512, 768) and k <= E.shape[0]:
            # the bf16 image and max||E|| are cached for a frozen E; the key carries the tensor's version, which
            # load_state_dict / copy_ bump. A trainable E is written in place by libhvae's Adam (no version bump),
            # so its image is rebuilt on every call
            key = (E.data_ptr(), tuple(E.shape), self.item_embeddings._version)
            cache = None if getattr(self, "item_embeddings_trainable", False) else getattr(self, "_topk_cache", None)
            if cache is None or cache[0] != key:
                E32 = E.contiguous()
                cache = (key, E32, ops.decoder_image(E32), ops.row_norm_max(E32))
                self._topk_cache = cache
            _, E32, img, emax = cache
            return ops.topk_fused(u, img, E32, emax, k, exclude=exclude)
        S = ops.gemm(u, E.t())
        return ops.topk(S, k, exclude=exclude)

    # -------------------------------------------------- fused eval path ---
    @torch.no_grad()
    def user_vectors(self, csr: ops.Csr, use_mean: bool = True) -> torch.Tensor:
        """u = projection(mu) for a CSR batch, eval mode (decode input of RecommendationEvaluator)."""
        was = self.training
        self.eval()
        try:
            mu, _ = self.encode(csr)
            return self.projection_layer(mu).contiguous()
        finally:
            self.train(was)


def vae_loss_function(
    recon_x: torch.Tensor,
    x: torch.Tensor,
    mu: torch.Tensor,
    logvar: torch.Tensor,
    beta: float = 0.2,
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """recon + beta * KL on materialised scores (reference: model.py:259-292), HIP kernels."""
    ops.require_hip(recon_x, x, mu, logvar)
    return VaeLossFn.apply(recon_x, x, mu, logvar, float(beta))


class AnnealedVAE(HybridVAE):
    """HybridVAE with a linear beta schedule (reference: model.py:295-334)."""

    def __init__(self, *args, **kwargs):
        self.beta_min = kwargs.pop("beta_min", 0.0)
        self.beta_max = kwargs.pop("beta_max", kwargs.get("beta", 0.2))
        self.anneal_steps = kwargs.pop("anneal_steps", 10000)
        super().__init__(*args, **kwargs)
        self.current_step = 0

    def get_current_beta(self) -> float:
        if self.current_step >= self.anneal_steps:
            return self.beta_max
        progress = self.current_step / self.anneal_steps
        return self.beta_min + progress * (self.beta_max - self.beta_min)

    def step_annealing(self):
        self.current_step += 1

    def compute_loss(self, recon_x, x, mu, logvar):
        return vae_loss_function(recon_x, x, mu, logvar, self.get_current_beta())


def create_hybrid_vae(
    n_items: int,
    item_embeddings: np.ndarray,
    latent_dim: int = 200,
    hidden_dims: Optional[list] = None,
    dropout: float = 0.5,
    beta: float = 0.2,
    use_annealing: bool = False,
    freeze_embeddings: bool = True,
    **annealing_kwargs,
) -> HybridVAE:
    """Factory (reference: model.py:337-385)."""
    if use_annealing:
        return AnnealedVAE(n_items=n_items, item_embeddings=item_embeddings, latent_dim=latent_dim,
                           hidden_dims=hidden_dims, dropout=dropout, beta=beta,
                           freeze_embeddings=freeze_embeddings, **annealing_kwargs)
    return HybridVAE(n_items=n_items, item_embeddings=item_embeddings, latent_dim=latent_dim,
                     hidden_dims=hidden_dims, dropout=dropout, beta=beta, freeze_embeddings=freeze_embeddings)
