"""The reference's processed-data artifacts -> CSR, without DataFrames (libhvae host loader).

Reference: load_training_data + _build_matrix + get_user_indices_from_df (src/ml/train.py:153-193). `mappings.pkl`
(the reference's own artifact, written by src/preprocessing/dataset.py:156-165) is still unpickled for its
user_to_idx / item_to_idx dicts; train.csv / val.csv are read by hvae_read_interactions in one native pass.
"""
from __future__ import annotations

import ctypes as C
import pickle
from pathlib import Path

import numpy as np
from scipy.sparse import csr_matrix

from ._lib import HostCsr, check, lib


def key_buffer(mapping: dict) -> tuple[bytes, int]:
    """The mapping's keys in index order as one NUL-separated buffer (key i <-> index i)."""
    keys = [None] * len(mapping)
    for k, i in mapping.items():
        keys[i] = k
    if any(k is None for k in keys):
        raise ValueError("mapping indices are not 0..n-1")
    text = "\0".join(str(k) for k in keys)
    buf = text.encode("utf-8")
    if buf.count(b"\0") != len(keys) - 1:
        raise ValueError("a mapping key contains a NUL character")
    return buf, len(keys)


class KeyBuffers:
    """user / item key buffers of one mappings dict, built once and reused for several files."""

    def __init__(self, mappings: dict):
        self.users, self.n_users = key_buffer(mappings["user_to_idx"])
        self.items, self.n_items = key_buffer(mappings["item_to_idx"])


def read_interactions(csv_path, keys: KeyBuffers, positives_only: bool = True) -> tuple[csr_matrix, list[int]]:
    """(CSR of the file's positives [n_users, n_items] with duplicates summed, the file's users in first-appearance
    order) -- _build_matrix(df, ...) and get_user_indices_from_df(df, ...) of the reference."""
    out = HostCsr()
    check(lib().hvae_read_interactions(str(csv_path).encode(), keys.users, len(keys.users), keys.n_users,
                                       keys.items, len(keys.items), keys.n_items, int(positives_only),
                                       C.byref(out)), "hvae_read_interactions")
    n, ncol, nnz = out.n_rows, out.n_cols, out.nnz
    try:
        rp = np.ctypeslib.as_array(C.cast(out.row_ptr, C.POINTER(C.c_int64)), shape=(n + 1,)).copy()
        ci = (np.ctypeslib.as_array(C.cast(out.col_idx, C.POINTER(C.c_int32)), shape=(nnz,)).copy()
              if nnz else np.zeros(0, np.int32))
        va = (np.ctypeslib.as_array(C.cast(out.vals, C.POINTER(C.c_float)), shape=(nnz,)).copy()
              if nnz else np.zeros(0, np.float32))
        users = (np.ctypeslib.as_array(C.cast(out.users, C.POINTER(C.c_int64)), shape=(out.n_users_seen,)).tolist()
                 if out.n_users_seen else [])
    finally:
        lib().hvae_host_csr_free(C.byref(out))
    m = csr_matrix((va, ci, rp), shape=(n, ncol))
    m.has_sorted_indices = True
    return m, users


def load_training_csr(data_dir: str):
    """train / val matrices and user lists of a processed data dir, plus the mappings dict and the matrix shape
    (len(user_to_idx), len(item_to_idx)) -- the shape the reference's interaction_matrix.pkl has
    (src/preprocessing/dataset.py:49-65), which is therefore not unpickled."""
    path = Path(data_dir)
    with open(path / "mappings.pkl", "rb") as f:
        mappings = pickle.load(f)  # the project's own dataset artifact
    keys = KeyBuffers(mappings)
    train, train_users = read_interactions(path / "train.csv", keys)
    val, val_users = read_interactions(path / "val.csv", keys)
    return (keys.n_users, keys.n_items), train, val, train_users, val_users, mappings
