"""Start-up cost of the data artifacts: the reference's pandas path against the native loader (hvae/io.py).

    python scripts/bench_loader.py [--users 1000000] [--per-user 20] [--dir /tmp/hvae_loader]

Writes a processed-data directory shaped like the reference's (src/preprocessing/dataset.py:141-170: train.csv /
val.csv with the review columns, mappings.pkl, interaction_matrix.pkl), then times, on the host:
  * reference: load_training_data (pickle the full matrix + mappings, pd.read_csv x 2) + _build_matrix x 2 +
    get_user_indices_from_df x 2 (src/ml/train.py:153-193, 216-226);
  * native: hvae.io.load_training_csr (mappings unpickled, each CSV one hvae_read_interactions pass).
Both results are compared for equality. Prints one JSON line.
"""
import argparse
import json
import pickle
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd")]


def write_dir(d: Path, n_users: int, per_user: int, n_items: int, seed: int = 0):
    import pandas as pd
    from scipy.sparse import csr_matrix
    d.mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(seed)
    users = np.char.add("A", np.char.zfill(np.arange(n_users).astype(str), 12))  # sorted = LabelEncoder order
    items = np.char.add("B0", np.char.zfill(np.arange(n_items).astype(str), 8))
    cnt = 5 + rng.poisson(per_user - 5, n_users)
    uidx = np.repeat(np.arange(n_users), cnt)
    iidx = (rng.zipf(1.3, uidx.size) - 1) % n_items
    n = uidx.size
    rating = rng.integers(1, 6, n)
    split = rng.random(n)
    df = pd.DataFrame({"rating": rating.astype(float), "title": "Great product, would buy",
                       "text": "Works as described.", "asin": items[iidx], "parent_asin": items[iidx],
                       "user_id": users[uidx], "timestamp": rng.integers(1_500_000_000_000, 1_700_000_000_000, n),
                       "verified_purchase": True, "binary_rating": (rating >= 4).astype(int)})
    df[split < 0.8].to_csv(d / "train.csv", index=False)
    df[(split >= 0.8) & (split < 0.9)].to_csv(d / "val.csv", index=False)
    u2i = {u: i for i, u in enumerate(users.tolist())}
    i2i = {it: i for i, it in enumerate(items.tolist())}
    with open(d / "mappings.pkl", "wb") as f:
        pickle.dump({"user_to_idx": u2i, "item_to_idx": i2i, "idx_to_user": {i: u for u, i in u2i.items()},
                     "idx_to_item": {i: it for it, i in i2i.items()}}, f)
    m = csr_matrix((df["binary_rating"].values.astype(np.float32), (uidx, iidx)), shape=(n_users, n_items))
    with open(d / "interaction_matrix.pkl", "wb") as f:
        pickle.dump(m, f)
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--per-user", type=int, default=20)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--dir", default="/tmp/hvae_loader")
    args = ap.parse_args()
    d = Path(args.dir)
    t = time.perf_counter()
    rows = write_dir(d, args.users, args.per_user, args.items)
    t_gen = time.perf_counter() - t
    from hvae import io as hio
    from src.ml.train import _build_matrix, get_user_indices_from_df, load_training_data

    t = time.perf_counter()
    full, train_df, val_df, mappings = load_training_data(str(d))
    u2i, i2i = mappings["user_to_idx"], mappings["item_to_idx"]
    tr = _build_matrix(train_df, u2i, i2i, full.shape)
    va = _build_matrix(val_df, u2i, i2i, full.shape)
    tru, vau = get_user_indices_from_df(train_df, u2i), get_user_indices_from_df(val_df, u2i)
    t_ref = time.perf_counter() - t
    del train_df, val_df, full

    t = time.perf_counter()
    shape, tr2, va2, tru2, vau2, _ = hio.load_training_csr(str(d))
    t_nat = time.perf_counter() - t

    same = True
    for a, b in ((tr, tr2), (va, va2)):
        a = a.tocsr()
        a.sum_duplicates()
        same &= bool(np.array_equal(a.indptr, b.indptr) and np.array_equal(a.indices, b.indices)
                     and np.array_equal(a.data.astype(np.float32), b.data))
    same &= tru == tru2 and vau == vau2
    csv_mb = ((d / "train.csv").stat().st_size + (d / "val.csv").stat().st_size) / 2 ** 20
    print(json.dumps({"users": args.users, "items": args.items, "rows": rows, "csv_MiB": round(csv_mb, 1),
                      "reference_pandas_s": round(t_ref, 2), "native_s": round(t_nat, 2),
                      "speedup": round(t_ref / t_nat, 1), "identical": same, "generate_s": round(t_gen, 1)}))


if __name__ == "__main__":
    main()
