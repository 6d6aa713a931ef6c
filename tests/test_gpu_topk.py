"""Fused exact top-K (hvae_topk_fused: bf16 MFMA shortlist + fp32 rescore, no [R, N] score matrix) against a
float64 ranking of the same fp32 inputs.

Reference semantics: RecommendationEvaluator.get_user_recommendations (src/ml/evaluate.py:137-147) and the
/recommend handler (src/api/server.py:115-183): scores = u E^T, seen items -> -inf, argsort descending, first
top_k. Indices must be identical except between items whose float64 scores are within fp32 rounding of each
other (the reference's own fp32 sgemm cannot order those either); returned scores equal the float64 score of the
returned item to 2e-6 relative."""
import numpy as np
import pytest
import torch

from gen import synth_csr, synth_embeddings

pytestmark = pytest.mark.gpu


def _case(hip_device, R, N, D, seed, scale=4.0):
    from hvae import ops
    E = torch.as_tensor(synth_embeddings(N, D, seed=seed))
    g = torch.Generator().manual_seed(seed + 1)
    U = torch.randn(R, D, generator=g) * (scale / D ** 0.5)
    Ed = E.to(hip_device)
    img = ops.decoder_image(Ed)
    emax = ops.row_norm_max(Ed)
    return U, E, U.to(hip_device), Ed, img, emax


def _check(idx, val, U, E, k, seen=None):
    S = U.double() @ E.double().t()
    if seen is not None:
        for r, items in enumerate(seen):
            S[r, items] = -np.inf
    idx = idx.cpu().long()
    val = val.cpu().double()
    tol = 2e-6 * S.abs().max().item()
    for r in range(S.shape[0]):
        order = sorted(range(S.shape[1]), key=lambda i: (-S[r, i].item(), -i))[:k] if S.shape[1] <= 4096 else None
        if order is None:
            top = torch.topk(S[r], k + 16)
            cand = sorted(zip(top.values.tolist(), top.indices.tolist()), key=lambda t: (-t[0], -t[1]))
            order = [i for _, i in cand[:k]]
        got = idx[r].tolist()
        assert len(set(got)) == k, r
        for j in range(k):
            if got[j] != order[j]:
                assert abs(S[r, got[j]].item() - S[r, order[j]].item()) <= tol, (r, j, got[j], order[j])
            assert abs(val[r, j].item() - S[r, got[j]].item()) <= tol, (r, j)
        if seen is not None:
            assert not set(got) & set(seen[r].tolist()), r


@pytest.mark.parametrize("R,N,D,k", [(64, 12101, 384, 10), (300, 100000, 384, 20), (37, 5003, 768, 50),
                                     (9, 2000, 128, 100), (130, 30011, 256, 10), (33, 777, 64, 5),
                                     (40, 20000, 512, 16)])
def test_topk_fused_exact(hip_device, R, N, D, k):
    from hvae import ops
    U, E, Ud, Ed, img, emax = _case(hip_device, R, N, D, seed=N + D)
    idx, val, flag = ops.topk_fused(Ud, img, Ed, emax, k, with_flags=True)
    assert int(flag.sum()) == 0  # the fused path certified every row itself
    _check(idx, val, U, E, k)


@pytest.mark.parametrize("R,N,D,k", [(64, 12101, 384, 10), (50, 40000, 768, 20)])
def test_topk_fused_exclude_seen(hip_device, R, N, D, k):
    """exclude_seen: K_u = k + |seen_u| shortlist, seen items removed before ranking (server.py:152-155)."""
    from hvae import ops
    U, E, Ud, Ed, img, emax = _case(hip_device, R, N, D, seed=7 * N)
    X = synth_csr(R, N, lam=15.0, seed=N)
    csr = ops.csr_from_scipy(X, hip_device)
    rows = torch.arange(R, dtype=torch.int32, device=hip_device)
    ex = ops.Csr(csr.row_ptr, csr.col_idx, csr.vals, N, rows=rows)
    idx, val, flag = ops.topk_fused(Ud, img, Ed, emax, k, exclude=ex, with_flags=True)
    assert int(flag.sum()) == 0
    seen = [torch.as_tensor(X[r].indices.astype(np.int64)) for r in range(R)]
    _check(idx, val, U, E, k, seen)
    # the same as the exact score-matrix path (hvae_gemm_f32 + hvae_topk)
    S = ops.gemm(Ud, Ed.t())
    i2, _ = ops.topk(S, k, exclude=ex)
    assert (idx.cpu() == i2.cpu()).float().mean() > 0.99


def test_topk_fused_flagged_rows_take_the_exact_path(hip_device):
    """Rows the fused kernel cannot certify (here: more seen items than the shortlist heap, and an all-seen row
    leaving fewer than k items) are flagged and ranked by the exact path; the answer stays exact."""
    from hvae import ops
    R, N, D, k = 6, 3000, 128, 8
    U, E, Ud, Ed, img, emax = _case(hip_device, R, N, D, seed=5)
    from scipy.sparse import csr_matrix
    rng = np.random.default_rng(0)
    rows_l, cols_l = [], []
    sizes = [3, 400, 0, 10, 2995, 260]  # row 1: 400 + k > 256 -> flagged; row 4: 5 unseen < k -> flagged
    for r, s in enumerate(sizes):
        c = rng.choice(N, s, replace=False)
        rows_l += [r] * s
        cols_l += c.tolist()
    X = csr_matrix((np.ones(len(rows_l), np.float32), (rows_l, cols_l)), shape=(R, N))
    csr = ops.csr_from_scipy(X, hip_device)
    ex = ops.Csr(csr.row_ptr, csr.col_idx, csr.vals, N, rows=torch.arange(R, dtype=torch.int32, device=hip_device))
    idx, val, flag = ops.topk_fused(Ud, img, Ed, emax, k, exclude=ex, with_flags=True)
    f = flag.cpu().tolist()
    assert f[1] == 1 and f[4] == 1 and f[5] == 1 and f[0] == 0 and f[2] == 0 and f[3] == 0
    X.sort_indices()
    seen = [torch.as_tensor(X[r].indices.astype(np.int64)) for r in range(R)]
    ok = [r for r in range(R) if r != 4]
    _check(idx[ok], val[ok], U[ok], E, k, [seen[r] for r in ok])
    # row 4 has 5 unseen items: those 5 first (exact order), then -inf
    S4 = (U[4].double() @ E.double().t())
    S4[seen[4]] = -np.inf
    top5 = sorted(range(N), key=lambda i: (-S4[i].item(), -i))[:5]
    assert idx[4, :5].cpu().tolist() == top5
    assert torch.isinf(val[4, 5:]).all()


@pytest.mark.parametrize("R,N,D,k", [(1, 200_000, 768, 10), (5, 20, 128, 5), (3, 50, 256, 50), (2, 31, 64, 7),
                                     (70, 4097, 384, 1)])
def test_topk_fused_edge_shapes(hip_device, R, N, D, k):
    """A single user over 200 K items, fewer items than one 32-item tile, k = N, a partial last tile, k = 1."""
    from hvae import ops
    U, E, Ud, Ed, img, emax = _case(hip_device, R, N, D, seed=3 * N + D)
    idx, val = ops.topk_fused(Ud, img, Ed, emax, k)
    _check(idx, val, U, E, k)


def test_topk_fused_exclusion_edges(hip_device):
    """Rows with nothing seen, and a row whose unseen items number exactly k."""
    from scipy.sparse import csr_matrix
    from hvae import ops
    R, N, D, k = 4, 600, 128, 6
    U, E, Ud, Ed, img, emax = _case(hip_device, R, N, D, seed=17)
    rows = [2] * (N - k) + [3, 3]
    cols = list(range(N - k)) + [7, 590]
    X = csr_matrix((np.ones(len(rows), np.float32), (rows, cols)), shape=(R, N))
    csr = ops.csr_from_scipy(X, hip_device)
    ex = ops.Csr(csr.row_ptr, csr.col_idx, csr.vals, N, rows=torch.arange(R, dtype=torch.int32, device=hip_device))
    idx, val = ops.topk_fused(Ud, img, Ed, emax, k, exclude=ex)
    X.sort_indices()
    seen = [torch.as_tensor(X[r].indices.astype(np.int64)) for r in range(R)]
    _check(idx, val, U, E, k, seen)
    assert sorted(idx[2].cpu().tolist()) == list(range(N - k, N))  # exactly the k unseen items
    R0 = ops.topk_fused(Ud[:0], img, Ed, emax, k)
    assert R0[0].shape == (0, k)


def test_topk_fused_bf16_midpoint_adversarial(hip_device):
    """the shortlist bound eps_u (hvae_topk.hip) must cover bf16 rounding of BOTH u and E. u's first
    half and the true top item's E row sit just below the bf16 rounding midpoint (both round down by ~2^-8), so
    the top item's bf16 score is ~2^-7 low; 40 competitors live on u's bf16-exact half with bf16-exact E, scoring
    just under the top in fp32 but ~0.49 above it in bf16, i.e. above the top by more than a 2^-8 bound (0.37)
    and less than the 2^-7 one (0.73). The fused top-K must still return the top item first, as the fp32 score
    matrix + hvae_topk do."""
    from hvae import ops
    N, D, k = 3000, 128, 10
    c = 1.0 + 2.0 ** -8 - 2.0 ** -20  # rounds down to 1.0 in bf16
    u = torch.ones(1, D, dtype=torch.float64)
    u[0, : D // 2] = c
    g = torch.Generator().manual_seed(5)
    E = torch.rand(N, D, generator=g, dtype=torch.float64) * 0.05  # the rest: far below
    E[0] = 0.0
    E[0, : D // 2] = c  # the true top: 64 c^2 = 64.4995 in fp32, 64 in bf16
    for j in range(1, 41):  # competitors: bf16-exact, on u's exact half, 64.43 .. 64.49 in both precisions
        E[j] = 0.0
        n_up = 55 + (j % 9)
        E[j, D // 2:] = 1.0
        E[j, D // 2: D // 2 + n_up] = 1.0078125
    U = u.float()
    Ef = E.float()
    S = U.double() @ Ef.double().t()
    assert int(S[0].argmax()) == 0 and S[0, 0] - S[0, 1:41].max() > 0
    Ud, Ed = U.to(hip_device), Ef.to(hip_device)
    img = ops.decoder_image(Ed)
    emax = ops.row_norm_max(Ed)
    bf = (U.bfloat16().double() @ Ef.bfloat16().double().t())[0]
    assert bf[1:41].min() - bf[0] > 0.37 * 1.02  # the 2^-8 bound would have dropped the top item
    idx, val, flag = ops.topk_fused(Ud, img, Ed, emax, k, with_flags=True)
    assert int(flag.sum()) == 0
    assert int(idx[0, 0]) == 0
    _check(idx, val, U, Ef, k)
    i2, _ = ops.topk(ops.gemm(Ud, Ed.t()), k)  # the exact score-matrix path
    assert idx.cpu().tolist() == i2.cpu().tolist()


@pytest.mark.timeout(300)
def test_topk_fused_extent_past_2gb(hip_device):
    """the bf16 image of 1.5 M items x d 768 is 2.3 GB, past the 2^31-byte extent one buffer
    resource addresses (hvae_topk.hip splits the sweep into extents with split-relative resources). 64 users must
    get the float64 ranking of the same fp32 inputs (or a clean HVAE_REQUIRE error, never a wrong answer)."""
    from hvae import ops
    R, N, D, k = 64, 1_500_000, 768, 20
    assert N * D * 2 >= 2 ** 31
    g = torch.Generator(device=hip_device).manual_seed(1234)
    Ed = torch.randn(N, D, generator=g, device=hip_device)
    Ed /= Ed.norm(dim=1, keepdim=True)
    # users aligned with items spread over the whole range (the last extent included) plus noise
    tgt = torch.linspace(0, N - 1, R, device=hip_device).long()
    Ud = (4.0 * Ed[tgt] + 0.5 * torch.randn(R, D, generator=g, device=hip_device) / D ** 0.5).contiguous()
    img = ops.decoder_image(Ed)
    emax = ops.row_norm_max(Ed)
    try:
        idx, val, flag = ops.topk_fused(Ud, img, Ed, emax, k, with_flags=True)
    except RuntimeError as e:  # the only acceptable failure: the library refuses the extent itself
        assert "extent" in str(e).lower() or "2^31" in str(e), e
        return
    torch.cuda.synchronize()
    # float64 reference on the device, in item chunks
    Ud64 = Ud.double()
    best_v = torch.full((R, k + 16), -float("inf"), dtype=torch.float64, device=hip_device)
    best_i = torch.zeros((R, k + 16), dtype=torch.long, device=hip_device)
    for s in range(0, N, 100_000):
        Sc = Ud64 @ Ed[s:s + 100_000].double().t()
        v, i = torch.topk(torch.cat([best_v, Sc], 1), k + 16, dim=1)
        best_i = torch.gather(torch.cat([best_i, torch.arange(s, s + Sc.shape[1], device=hip_device).expand(R, -1)],
                                        1), 1, i)
        best_v = v
    gi, gv = idx.long(), val.double()
    tol = 2e-6 * best_v[:, 0].abs().max().item()
    for r in range(R):
        cand = sorted(zip(best_v[r].tolist(), best_i[r].tolist()), key=lambda t: (-t[0], -t[1]))[:k]
        for j in range(k):
            got = int(gi[r, j])
            if got != cand[j][1]:
                assert abs(cand[j][0] - (Ud64[r] @ Ed[got].double()).item()) <= tol, (r, j, got, cand[j])
            assert abs(gv[r, j].item() - (Ud64[r] @ Ed[got].double()).item()) <= tol, (r, j)
    assert (gi[:, 0] == tgt).float().mean() > 0.9  # the planted item leads (sanity of the construction)
