"""Native data-artifact loader (hvae_read_interactions, host code in libhvae) against the pandas path of the
reference (load_training_data + _build_matrix + get_user_indices_from_df, src/ml/train.py:153-193; the pandas
functions here are pinned to the reference's behaviour by golden G5 in test_api_cpu.py). Runs on CPU."""
import pickle

import numpy as np
import pandas as pd
import pytest


def _write_dir(tmp_path, n_users=300, n_items=120, rows=4000, seed=0):
    rng = np.random.default_rng(seed)
    users = [f"U{rng.integers(1e9):09d}x" for _ in range(n_users)]
    items = [f"B0{rng.integers(1e8):08d}" for _ in range(n_items)]
    users, items = sorted(set(users)), sorted(set(items))  # LabelEncoder classes_ order
    u2i = {u: i for i, u in enumerate(users)}
    i2i = {it: i for i, it in enumerate(items)}
    titles = ["plain", "with, comma", 'a "quoted" word', "two\nlines", "", "trailing,\"mixed\", \"stuff\"\r\nx"]

    def frame(n, s):
        r = np.random.default_rng(s)
        return pd.DataFrame({
            "user_id": [users[j] for j in r.integers(len(users), size=n)],
            "asin": [items[j] for j in r.zipf(1.5, size=n) % len(items)],  # heavy duplicates
            "title": [titles[j] for j in r.integers(len(titles), size=n)],
            "rating": r.integers(1, 6, size=n).astype(float),
            "binary_rating": (r.random(n) < 0.7).astype(int),
            "timestamp": r.integers(1_500_000_000, 1_700_000_000, size=n),
        })

    train, val = frame(rows, seed + 1), frame(rows // 8, seed + 2)
    # a user that appears only in non-positive rows, and one with no rows at all
    extra = pd.DataFrame({"user_id": [users[0]], "asin": [items[1]], "title": ["x"], "rating": [1.0],
                          "binary_rating": [0], "timestamp": [1]})
    val = pd.concat([extra, val], ignore_index=True)
    train.to_csv(tmp_path / "train.csv", index=False)  # as src/preprocessing/dataset.py:149-150 writes them
    val.to_csv(tmp_path / "val.csv", index=False)
    with open(tmp_path / "mappings.pkl", "wb") as f:
        pickle.dump({"user_to_idx": u2i, "item_to_idx": i2i, "idx_to_user": {i: u for u, i in u2i.items()},
                     "idx_to_item": {i: it for it, i in i2i.items()}}, f)
    return u2i, i2i


def test_native_loader_equals_pandas_path(tmp_path):
    from hvae import io as hio
    from src.ml.train import _build_matrix, get_user_indices_from_df
    u2i, i2i = _write_dir(tmp_path)
    shape, train, val, train_users, val_users, mappings = hio.load_training_csr(str(tmp_path))
    assert shape == (len(u2i), len(i2i))
    for name, got, got_users in (("train", train, train_users), ("val", val, val_users)):
        df = pd.read_csv(tmp_path / f"{name}.csv", low_memory=False)
        ref = _build_matrix(df, u2i, i2i, shape).tocsr()
        ref.sum_duplicates()
        ref.sort_indices()
        np.testing.assert_array_equal(got.indptr, ref.indptr)
        np.testing.assert_array_equal(got.indices, ref.indices)
        np.testing.assert_array_equal(got.data, ref.data.astype(np.float32))
        assert got_users == get_user_indices_from_df(df, u2i), name


def test_native_loader_without_binary_column_and_errors(tmp_path):
    from hvae import io as hio
    u2i, i2i = _write_dir(tmp_path, rows=500)
    df = pd.read_csv(tmp_path / "train.csv")
    df.drop(columns=["binary_rating"]).to_csv(tmp_path / "nobin.csv", index=False)
    keys = hio.KeyBuffers({"user_to_idx": u2i, "item_to_idx": i2i})
    m, users = hio.read_interactions(tmp_path / "nobin.csv", keys)
    # without the column every row is a positive (reference: `if "binary_rating" in df.columns`)
    assert m.sum() == len(df)
    bad = df.copy()
    bad.loc[3, "asin"] = "NOT_AN_ITEM"
    bad.loc[3, "binary_rating"] = 1
    bad.to_csv(tmp_path / "bad.csv", index=False)
    with pytest.raises(RuntimeError, match="do not know"):
        hio.read_interactions(tmp_path / "bad.csv", keys)
    bad.loc[3, "binary_rating"] = 0  # unknown item on a non-positive row: never indexed, fine
    bad.to_csv(tmp_path / "bad.csv", index=False)
    m2, _ = hio.read_interactions(tmp_path / "bad.csv", keys)
    assert m2.nnz > 0
