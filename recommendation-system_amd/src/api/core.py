"""The /recommend and /recommend/batch compute on MI355X, without the web layer.

Reference: src/api/server.py:115-183 (`get_recommendations`: user vector from the interaction matrix ->
get_user_embedding -> decode -> seen items to -inf -> argsort descending -> the first top_k with finite scores,
mapped through idx_to_item), :264-299 (`get_batch_recommendations`: at most 100 users, per-user errors in the
result), :300-358 (`load_model_and_data`). The FastAPI app, its schemas and the Streamlit UI stay out of scope
(DESIGN.md §7); a maintainer keeps the reference's handlers and calls RecommendationCore from them
(INTEGRATION.md).

A batch is one device pass: the users' CSR rows are read in place (no dense [B, N] vectors), u = projection(mu)
for all of them in one encoder launch, and the fused exact top-K (hvae_topk_fused) ranks them against E without
forming the [B, N] score matrix.
"""
from __future__ import annotations

import pickle
from pathlib import Path

import numpy as np
import torch
from scipy.sparse import csr_matrix

from hvae import ops

from ..ml.evaluate import load_model_from_checkpoint
from ..ml.model import HybridVAE
from ..preprocessing.embeddings import load_embeddings

MAX_BATCH = 100  # server.py:283
MAX_TOP_K = 100  # schemas.py:8 (RecommendationRequest.top_k: 1 <= top_k <= 100)


class UserNotFound(KeyError):
    """The reference answers 404 "User '<id>' not found in training data" (server.py:131-135)."""


class RecommendationCore:
    def __init__(self, model: HybridVAE, interaction_matrix: csr_matrix, user_to_idx: dict, item_to_idx: dict,
                 idx_to_item: dict, device: torch.device):
        if device.type != "cuda":
            raise RuntimeError("RecommendationCore runs on the MI355X HIP device only")
        self.model = model.to(device).eval()
        self.device = device
        self.interaction_matrix = interaction_matrix.tocsr()
        self.user_to_idx, self.item_to_idx, self.idx_to_item = user_to_idx, item_to_idx, idx_to_item
        self.n_items = self.interaction_matrix.shape[1]
        self._csr = ops.csr_from_scipy(self.interaction_matrix, device)

    @classmethod
    def from_artifacts(cls, model_path: str, data_dir: str, embeddings_path: str,
                       device_name: str = "cuda") -> "RecommendationCore":
        """load_model_and_data (server.py:300-358): interaction_matrix.pkl, mappings.pkl (the reference's own
        processed-data artifacts), the embeddings file and a checkpoint."""
        if device_name not in ("cuda", None) or not torch.cuda.is_available():
            raise RuntimeError("the MI355X recommendation core needs the HIP device (device 'cuda')")
        device = torch.device("cuda", torch.cuda.current_device())
        data_path = Path(data_dir)
        with open(data_path / "interaction_matrix.pkl", "rb") as f:
            interaction_matrix = pickle.load(f)
        with open(data_path / "mappings.pkl", "rb") as f:
            mappings = pickle.load(f)
        embeddings, _, _ = load_embeddings(embeddings_path)
        model = load_model_from_checkpoint(model_path, embeddings, device)
        return cls(model, interaction_matrix, mappings["user_to_idx"], mappings["item_to_idx"],
                   mappings["idx_to_item"], device)

    # ------------------------------------------------------------ device core --
    @torch.no_grad()
    def recommend_indices(self, user_idx, top_k: int = 10, exclude_seen: bool = True):
        """Item indices [n, top_k] (int64) and fp32 scores [n, top_k] for user rows `user_idx`, in the
        reference's order (score descending; excluded items score -inf and sort last)."""
        users = np.asarray(user_idx, np.int32).reshape(-1)
        if len(users) == 0:
            return np.zeros((0, top_k), np.int64), np.zeros((0, top_k), np.float32)
        rows = torch.as_tensor(users, device=self.device)
        csr = ops.Csr(self._csr.row_ptr, self._csr.col_idx, self._csr.vals, self.n_items, rows=rows)
        u = self.model.user_vectors(csr)
        k = min(top_k, self.n_items)
        idx, val = self.model.topk_scores(u, k, exclude=csr if exclude_seen else None)
        return idx.cpu().numpy().astype(np.int64), val.cpu().numpy()

    # ------------------------------------------------------------- reference API --
    def _items(self, idx_row, val_row) -> list[dict]:
        return [{"item_id": self.idx_to_item[int(i)], "score": float(s)}
                for i, s in zip(idx_row, val_row) if int(i) in self.idx_to_item and not np.isinf(s)]

    @staticmethod
    def _check_k(top_k: int):
        if not 1 <= int(top_k) <= MAX_TOP_K:
            raise ValueError(f"top_k must be in [1, {MAX_TOP_K}]")

    def recommend(self, user_id: str, top_k: int = 10, exclude_seen: bool = True) -> dict:
        """RecommendationResponse of POST /recommend as a dict: user_id, recommendations [{item_id, score}],
        total_items."""
        self._check_k(top_k)
        if user_id not in self.user_to_idx:
            raise UserNotFound(f"User '{user_id}' not found in training data")
        idx, val = self.recommend_indices([self.user_to_idx[user_id]], top_k, exclude_seen)
        return {"user_id": user_id, "recommendations": self._items(idx[0], val[0]),
                "total_items": len(self.item_to_idx)}

    def recommend_batch(self, user_ids: list[str], top_k: int = 10, exclude_seen: bool = True) -> dict:
        """POST /recommend/batch: {user_id: [items] | {"error": detail}}, at most 100 users; the known users are
        ranked in ONE device pass (the reference loops over them)."""
        if len(user_ids) > MAX_BATCH:
            raise ValueError(f"Maximum {MAX_BATCH} users per batch request")
        self._check_k(top_k)
        known = [uid for uid in user_ids if uid in self.user_to_idx]
        idx, val = self.recommend_indices([self.user_to_idx[u] for u in known], top_k, exclude_seen)
        pos = {u: i for i, u in enumerate(known)}
        out = {}
        for uid in user_ids:
            if uid in pos:
                out[uid] = self._items(idx[pos[uid]], val[pos[uid]])
            else:
                out[uid] = {"error": f"User '{uid}' not found in training data"}
        return out
