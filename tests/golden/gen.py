"""Deterministic synthetic inputs shared by the golden generator and the tests.

Rows follow SURVEY §8(d): nnz_u = 5 + Poisson(lam) item draws per user, item
ids drawn with replacement from Zipf p_i ~ (i+1)^-0.8, duplicates summed into
the values (as scipy does in src/ml/train.py:182). E ~ N(0, 1) rows,
L2-normalised (as src/preprocessing/embeddings.py:62). numpy PCG64 seeds.
"""
from __future__ import annotations

import hashlib

import numpy as np
from scipy.sparse import csr_matrix


def synth_csr(n_users: int, n_items: int, lam: float = 3.0, seed: int = 0, zipf: float = 0.8) -> csr_matrix:
    rng = np.random.Generator(np.random.PCG64(seed))
    p = (np.arange(n_items) + 1.0) ** (-zipf)
    p /= p.sum()
    counts = 5 + rng.poisson(lam, size=n_users)
    rows = np.repeat(np.arange(n_users), counts)
    cols = rng.choice(n_items, size=int(counts.sum()), p=p)
    m = csr_matrix((np.ones(len(rows), dtype=np.float64), (rows, cols)), shape=(n_users, n_items))
    m.sum_duplicates()
    return m


def synth_embeddings(n_items: int, d: int, seed: int = 1) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    e = rng.standard_normal((n_items, d)).astype(np.float32)
    return e / np.linalg.norm(e, axis=1, keepdims=True)


def synth_masks(shapes: list[tuple[int, int]], p: float, seed: int) -> list[np.ndarray]:
    """Dropout multipliers (0 or 1/(1-p)) for explicit-randomness parity."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for s in shapes:
        keep = rng.random(s) >= p
        out.append((keep / (1.0 - p)).astype(np.float32) if p < 1 else np.zeros(s, np.float32))
    return out


def synth_eps(shape: tuple[int, int], seed: int) -> np.ndarray:
    return np.random.Generator(np.random.PCG64(seed)).standard_normal(shape).astype(np.float32)


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()[:16]


# Configurations of the golden train-step fixtures (G2).
TRAIN_CONFIGS = {
    # projection MLP present (L != d), one hidden layer, dropout masks injected
    "A": dict(n_users=32, n_items=300, d=128, latent=64, hidden=[128], dropout=0.3, beta=0.2, lr=1e-3, seed=11),
    # identity projection (L == d), two hidden layers
    "B": dict(n_users=16, n_items=200, d=32, latent=32, hidden=[64, 48], dropout=0.5, beta=0.1, lr=1e-3, seed=12),
    # no dropout, heavier rows (duplicates -> values >= 2), weight decay
    "C": dict(n_users=8, n_items=150, d=64, latent=32, hidden=[64], dropout=0.0, beta=0.2, lr=2e-3, seed=13,
              wd=1e-4, lam=12.0),
}

# Eval-forward fixture (G1): Appliances-shaped items (890), best-config-like widths.
EVAL_CONFIG = dict(n_users=64, n_items=890, d=384, latent=64, hidden=[512], beta=0.2, seed=0)


# NDCG statistical fixture (G7): All_Beauty-shaped planted-cluster dataset (SURVEY §8c, G6 there).
PLANTED_CONFIG = dict(n_users=22363, n_items=12101, d=384, n_clusters=64, lam=3.0, p_home=0.7, noise=0.6,
                      seed=2024, latent=128, hidden=[512], dropout=0.3, beta=0.2, lr=1e-3, batch=64, epochs=20,
                      neg_seed=1234)


def synth_planted(n_users: int, n_items: int, d: int, n_clusters: int = 64, lam: float = 3.0,
                  p_home: float = 0.7, noise: float = 0.6, seed: int = 2024, **_):
    """Leave-one-out splits of a planted-cluster interaction log plus its item embeddings.

    Items are dealt to clusters; E_i = normalise(centroid(c_i) + noise * N(0, I/d)),
    so the frozen decoder can separate clusters. Each user has a home cluster and
    5 + Poisson(lam) distinct items, each from the home cluster with prob p_home,
    otherwise Zipf(0.8)-popular over all items. Per user (in draw order) the last item
    is the test positive, the one before it the val positive, the rest train
    (the reference's leave-one-out layout: data/{train,val,test}.csv, binary_rating 1).
    Returns (train_df, val_df, test_df, E [N, d] fp32, user_ids, item_ids).
    """
    import pandas as pd
    rng = np.random.Generator(np.random.PCG64(seed))
    cl = rng.permutation(n_items) % n_clusters
    cent = rng.standard_normal((n_clusters, d)).astype(np.float32) / np.sqrt(d)
    e = cent[cl] + noise * rng.standard_normal((n_items, d)).astype(np.float32) / np.sqrt(d)
    e = (e / np.linalg.norm(e, axis=1, keepdims=True)).astype(np.float32)
    members = [np.flatnonzero(cl == c) for c in range(n_clusters)]
    pop = (np.arange(n_items) + 1.0) ** -0.8
    pop /= pop.sum()
    home = rng.integers(0, n_clusters, size=n_users)
    counts = 5 + rng.poisson(lam, size=n_users)
    users, items, split = [], [], []
    for u in range(n_users):
        n = int(counts[u])
        seen: list[int] = []
        sset: set[int] = set()
        while len(seen) < n:
            i = int(rng.choice(members[home[u]])) if rng.random() < p_home else int(rng.choice(n_items, p=pop))
            if i not in sset:
                sset.add(i)
                seen.append(i)
        users += [u] * n
        items += seen
        split += [0] * (n - 2) + [1, 2]
    users, items, split = np.array(users), np.array(items), np.array(split)
    uid = np.array([f"U{u:07d}" for u in range(n_users)])
    iid = np.array([f"I{i:07d}" for i in range(n_items)])
    df = pd.DataFrame({"user_id": uid[users], "asin": iid[items], "rating": 5.0, "binary_rating": 1})
    return (df[split == 0].reset_index(drop=True), df[split == 1].reset_index(drop=True),
            df[split == 2].reset_index(drop=True), e, uid, iid)


def write_planted_artifacts(root, cfg: dict | None = None):
    """Write the reference's on-disk contract for the planted dataset under root:
    data/{train,val,test}.csv, data/interaction_matrix.pkl, data/mappings.pkl,
    embeddings/item_embeddings.npy (+ _mappings.pkl). Returns (data_dir, emb_path)."""
    import pickle
    from pathlib import Path
    cfg = dict(PLANTED_CONFIG, **(cfg or {}))
    root = Path(root)
    tr, va, te, E, uid, iid = synth_planted(**cfg)
    data, emb = root / "data", root / "embeddings"
    data.mkdir(parents=True, exist_ok=True)
    emb.mkdir(parents=True, exist_ok=True)
    tr.to_csv(data / "train.csv", index=False)
    va.to_csv(data / "val.csv", index=False)
    te.to_csv(data / "test.csv", index=False)
    u2i = {u: k for k, u in enumerate(uid)}
    i2i = {i: k for k, i in enumerate(iid)}
    import pandas as pd
    full = pd.concat([tr, va, te])
    mat = csr_matrix((np.ones(len(full)), (full["user_id"].map(u2i), full["asin"].map(i2i))),
                     shape=(len(uid), len(iid)))
    with open(data / "interaction_matrix.pkl", "wb") as f:
        pickle.dump(mat, f)
    with open(data / "mappings.pkl", "wb") as f:
        pickle.dump({"user_to_idx": u2i, "item_to_idx": i2i, "idx_to_user": dict(enumerate(uid)),
                     "idx_to_item": dict(enumerate(iid))}, f)
    np.save(emb / "item_embeddings.npy", E)
    with open(emb / "item_embeddings_mappings.pkl", "wb") as f:
        pickle.dump({"item_to_idx": i2i, "idx_to_item": dict(enumerate(iid))}, f)
    return data, emb / "item_embeddings.npy"
