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
