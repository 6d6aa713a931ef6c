"""The /recommend core (src/api/core.py) against the reference handler's own steps (src/api/server.py:115-183,
264-299) run through the module API: dense user vector -> get_user_embedding -> decode -> seen to -inf ->
np.argsort(scores)[::-1][:top_k], finite scores only, idx_to_item mapping."""
import numpy as np
import pytest
import torch

from gen import synth_csr, synth_embeddings

pytestmark = pytest.mark.gpu


@pytest.fixture
def core(hip_device):
    from src.api.core import RecommendationCore
    from src.ml.model import HybridVAE
    n_users, n_items = 150, 2000
    X = synth_csr(n_users, n_items, lam=6.0, seed=41)
    E = synth_embeddings(n_items, 384, seed=42)
    torch.manual_seed(3)
    model = HybridVAE(n_items, E, latent_dim=64, hidden_dims=[256], dropout=0.3, beta=0.2).to(hip_device)
    users = {f"user_{i}": i for i in range(n_users)}
    items = {f"item_{j}": j for j in range(n_items)}
    return RecommendationCore(model, X, users, items, {j: k for k, j in items.items()}, hip_device)


def _handler(core, user_id, top_k, exclude_seen):
    """The reference handler's computation, step by step, on the module API (pinned to golden G1)."""
    m = core.model
    uidx = core.user_to_idx[user_id]
    x = torch.as_tensor(core.interaction_matrix[uidx].toarray().flatten(), dtype=torch.float32,
                        device=core.device).unsqueeze(0)
    with torch.no_grad():
        scores = m.decode(m.get_user_embedding(x)).squeeze().double().cpu().numpy()
    if exclude_seen:
        scores[core.interaction_matrix[uidx].nonzero()[1]] = -np.inf
    top = np.argsort(scores, kind="stable")[::-1][:top_k]
    return scores, [(core.idx_to_item[int(i)], float(scores[i])) for i in top if not np.isinf(scores[i])]


@pytest.mark.parametrize("exclude_seen", [True, False])
def test_recommend_matches_handler(core, exclude_seen):
    for uid in ["user_0", "user_17", "user_149"]:
        got = core.recommend(uid, top_k=10, exclude_seen=exclude_seen)
        assert got["user_id"] == uid and got["total_items"] == 2000
        scores, ref = _handler(core, uid, 10, exclude_seen)
        tol = 2e-5 * np.abs(scores[np.isfinite(scores)]).max()
        assert len(got["recommendations"]) == len(ref)
        for g, (rid, rs) in zip(got["recommendations"], ref):
            gi = int(g["item_id"].split("_")[1])
            # identical items except where the scores tie within fp32 rounding
            assert g["item_id"] == rid or abs(scores[gi] - rs) <= tol
            assert abs(g["score"] - scores[gi]) <= tol


def test_recommend_batch_semantics(core):
    from src.api.core import UserNotFound
    out = core.recommend_batch(["user_3", "nobody", "user_4"], top_k=5)
    assert list(out) == ["user_3", "nobody", "user_4"]
    assert out["nobody"] == {"error": "User 'nobody' not found in training data"}
    for uid in ("user_3", "user_4"):
        single = core.recommend(uid, top_k=5)["recommendations"]
        assert out[uid] == single  # one batched pass = the per-user answers
    with pytest.raises(UserNotFound):
        core.recommend("nobody")
    with pytest.raises(ValueError):
        core.recommend_batch([f"user_{i}" for i in range(101)])
    with pytest.raises(ValueError):
        core.recommend("user_1", top_k=0)


def test_module_recommend_is_exact(core):
    """HybridVAE.recommend (reference model.py:236-256: torch.topk(decode(z), k)) through the fused top-K."""
    m = core.model
    g = torch.Generator().manual_seed(9)
    z = torch.randn(7, 64, generator=g).to(core.device)
    idx, val = m.recommend(z, top_k=25)
    with torch.no_grad():
        S = m.decode(z).double().cpu()
    tol = 2e-5 * S.abs().max().item()
    for r in range(7):
        ref = torch.topk(S[r], 25)
        for j in range(25):
            i = int(idx[r, j])
            assert i == int(ref.indices[j]) or abs(S[r, i].item() - ref.values[j].item()) <= tol
            assert abs(val[r, j].item() - S[r, i].item()) <= tol


def _topk_gemm(m, z, k):
    """The exact score-matrix path on the module's current E: fp32 hvae_gemm_f32 + hvae_topk."""
    from hvae import ops
    with torch.no_grad():
        u = m.projection_layer(z).contiguous()
        S = ops.gemm(u, m.item_embeddings.detach().t())
        return ops.topk(S, k)


def test_recommend_after_new_embeddings(core):
    """The fused top-K caches E's bf16 image keyed on the buffer's version (src/ml/model.py topk_scores): a
    recommend -> load_state_dict with another embedding file -> recommend must rank against the NEW E, as
    gemm + hvae_topk do (reference model.py:236-256 reads self.item_embeddings on every call). Then once more
    through an in-place copy_ of E."""
    from src.ml.model import HybridVAE
    m = core.model
    g = torch.Generator().manual_seed(11)
    z = torch.randn(9, 64, generator=g).to(core.device)
    i0, _ = m.recommend(z, top_k=20)
    r0, _ = _topk_gemm(m, z, 20)
    assert (i0.cpu() == r0.cpu().long()).float().mean() > 0.99
    E2 = synth_embeddings(2000, 384, seed=77)
    torch.manual_seed(3)  # same weights, other embeddings: only E changes
    other = HybridVAE(2000, E2, latent_dim=64, hidden_dims=[256], dropout=0.3, beta=0.2)
    m.load_state_dict(other.state_dict())
    i1, v1 = m.recommend(z, top_k=20)
    r1, s1 = _topk_gemm(m, z, 20)
    assert not torch.equal(i1.cpu(), i0.cpu())  # the ranking moved with E
    assert (i1.cpu() == r1.cpu().long()).float().mean() > 0.99
    torch.testing.assert_close(v1.cpu(), s1.cpu(), rtol=2e-5, atol=2e-5)
    with torch.no_grad():
        m.item_embeddings.copy_(torch.as_tensor(synth_embeddings(2000, 384, seed=78), device=core.device))
    i2, v2 = m.recommend(z, top_k=20)
    r2, s2 = _topk_gemm(m, z, 20)
    assert (i2.cpu() == r2.cpu().long()).float().mean() > 0.99
    torch.testing.assert_close(v2.cpu(), s2.cpu(), rtol=2e-5, atol=2e-5)
