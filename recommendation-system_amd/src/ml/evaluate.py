"""Evaluation on MI355X -- drop-in for the reference's src/ml/evaluate.py.

Same metrics, protocols, evaluator API, checkpoint loader and CLI as the
reference (src/ml/evaluate.py:32-374). The per-test-row Python loop with a
1 x N decode per row (:187-215) becomes batched device work: user vectors for
a batch of test rows through the HIP encoder, then either the 100 candidate
scores per row (99-negative protocol; hvae_score_candidates + hvae_rank_first)
or the full fp32 score matrix + exact top-K with seen items masked
(full-ranking protocol; hvae_gemm_f32 + hvae_topk). Negatives are drawn with
np.random.choice(available, n, replace=False) exactly as the reference does
(:159-170) -- draw for draw from numpy's global stream, by a native sampler over all rows at once
(hvae_negatives_legacy) -- so the negatives are the reference's.
"""
from __future__ import annotations

import argparse
import json
import logging
from pathlib import Path

import numpy as np
import pandas as pd
import torch
from scipy.sparse import csr_matrix

from hvae import ops
from hvae.dist import all_reduce_host, broadcast_seed, init_from_env, is_main

from ..config import config
from ..preprocessing.embeddings import load_embeddings
from .model import HybridVAE, create_hybrid_vae
from .train import load_training_data

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger(__name__)


# =============================================================================
# Metrics (reference: evaluate.py:32-54)
# =============================================================================


def recall_at_k(recommended: np.ndarray, relevant: np.ndarray, k: int) -> float:
    if len(relevant) == 0:
        return 0.0
    hits = len(np.intersect1d(recommended[:k], relevant))
    return hits / len(relevant)


def ndcg_at_k(recommended: np.ndarray, relevant: np.ndarray, k: int) -> float:
    if len(relevant) == 0:
        return 0.0
    dcg = sum(1.0 / np.log2(i + 2) for i, item in enumerate(recommended[:k]) if item in relevant)
    idcg = sum(1.0 / np.log2(i + 2) for i in range(min(len(relevant), k)))
    return dcg / idcg if idcg > 0 else 0.0


def hit_ratio_at_k(recommended: np.ndarray, relevant: np.ndarray, k: int) -> float:
    if len(relevant) == 0:
        return 0.0
    return 1.0 if len(np.intersect1d(recommended[:k], relevant)) > 0 else 0.0


def metrics_from_rank(rank: np.ndarray, k_values: list[int]) -> dict[int, dict[str, np.ndarray]]:
    """Per-row metrics for ONE relevant item at 0-based `rank` (vectorised form of the above)."""
    out = {}
    for k in k_values:
        hit = (rank < k).astype(np.float64)
        out[k] = {"recall": hit, "ndcg": np.where(rank < k, 1.0 / np.log2(rank + 2.0), 0.0), "hit_ratio": hit}
    return out


# =============================================================================
# Helpers
# =============================================================================


def _get_device(device: str | None = None) -> torch.device:
    if device:
        dev = torch.device(device)
        if dev.type != "cuda":  # the reference's cpu / mps choices parse, then fail here, before any data loads
            raise RuntimeError(f"device {device!r}: the MI355X HybridVAE path runs on a HIP device only; "
                               "there is no CPU fallback.")
        return dev
    if torch.cuda.is_available():
        return torch.device("cuda")
    raise RuntimeError("The MI355X HybridVAE path needs a HIP device; there is no CPU fallback.")


def _build_input_matrix(train_df: pd.DataFrame, val_df: pd.DataFrame, user_to_idx: dict, item_to_idx: dict,
                        shape: tuple) -> csr_matrix:
    """Train + val positives (reference: evaluate.py:73-87)."""
    train_pos = train_df[train_df["binary_rating"] == 1] if "binary_rating" in train_df.columns else train_df
    val_pos = val_df[val_df["binary_rating"] == 1] if "binary_rating" in val_df.columns else val_df
    combined = pd.concat([train_pos, val_pos])
    rows = combined["user_id"].map(user_to_idx)
    cols = combined["asin"].map(item_to_idx)
    return csr_matrix((np.ones(len(combined)), (rows, cols)), shape=shape)


_METRICS = ["recall", "ndcg", "hit_ratio"]


def _aggregate_metrics(all_metrics: dict, k_values: list[int], group=None, device=None) -> dict[int, dict[str, float]]:
    """Means of the per-row metrics (reference: evaluate.py:90-98). With a process group every rank holds a
    shard of the rows: the sums and the row count are all-reduced, so every rank returns the global means."""
    if group is None:
        return {
            k: {m: float(np.mean(all_metrics[k][m])) if len(all_metrics[k][m]) else 0.0 for m in _METRICS}
            for k in k_values
        }
    sums = [float(np.sum(all_metrics[k][m])) for k in k_values for m in _METRICS]
    n = len(all_metrics[k_values[0]]["recall"]) if k_values else 0
    tot = all_reduce_host(sums + [n], group, device)
    cnt = tot[-1]
    it = iter(tot[:-1])
    return {k: {m: (float(next(it)) / cnt if cnt else 0.0) for m in _METRICS} for k in k_values}


# =============================================================================
# Evaluator
# =============================================================================


class RecommendationEvaluator:
    """Leave-one-out evaluator (reference: evaluate.py:106-265), batched on the device."""

    def __init__(self, model: HybridVAE, interaction_matrix: csr_matrix, user_to_idx: dict[str, int],
                 item_to_idx: dict[str, int], device: torch.device, batch_size: int = 1024, process_group=None):
        """process_group: the dataset protocols shard their rows over its ranks (rank r scores rows r, r + W,
        ...) and all-reduce the metric sums; the 99-negative protocol first seeds numpy identically on every
        rank (from rank 0's global RNG) so that all ranks draw the same negatives for every row."""
        self.group = process_group
        self.model = model.to(device)
        self.model.eval()
        self.device = device
        self.interaction_matrix = interaction_matrix.tocsr()
        self.user_to_idx = user_to_idx
        self.item_to_idx = item_to_idx
        self.n_items = interaction_matrix.shape[1]
        self.batch_size = batch_size
        self._csr = ops.csr_from_scipy(self.interaction_matrix, device)
        self._E = self.model.item_embeddings.detach().contiguous()

    # ---- device helpers
    def _user_vectors(self, users: np.ndarray) -> torch.Tensor:
        rows = torch.as_tensor(np.asarray(users, np.int32), device=self.device)
        csr = ops.Csr(self._csr.row_ptr, self._csr.col_idx, self._csr.vals, self.n_items, rows=rows)
        return self.model.user_vectors(csr)

    def _scores(self, users: np.ndarray) -> torch.Tensor:
        """fp32 [len(users), N] scores = decode(get_user_embedding(x)) (reference: evaluate.py:125-135)."""
        u = self._user_vectors(users)
        return ops.gemm(u, self._E.t())

    # ---- reference per-user API
    def _get_user_scores(self, user_idx: int) -> np.ndarray:
        with torch.no_grad():
            return self._scores(np.array([user_idx]))[0].cpu().numpy()

    def get_user_recommendations(self, user_idx: int, top_k: int = 100, exclude_seen: bool = True):
        idx, val = self._topk(np.array([user_idx]), top_k, exclude_seen)
        return idx[0], val[0]

    def _topk(self, users: np.ndarray, k: int, exclude_seen: bool = True):
        """Top-k of a batch of users over all items (seen ones excluded): the fused top-K, no [B, N] scores."""
        with torch.no_grad():
            u = self._user_vectors(users)
            excl = None
            if exclude_seen:
                rows = torch.as_tensor(np.asarray(users, np.int32), device=self.device)
                excl = ops.Csr(self._csr.row_ptr, self._csr.col_idx, self._csr.vals, self.n_items, rows=rows)
            idx, val = self.model.topk_scores(u, k, exclude=excl)
        return idx.cpu().numpy().astype(np.int64), val.cpu().numpy()

    def evaluate_user_with_negatives(self, user_idx: int, test_item_idx: int, n_negatives: int = 99,
                                     k_values: list[int] | None = None) -> dict[int, dict[str, float]]:
        k_values = k_values or [5, 10, 20]
        negs = self._sample_negatives(user_idx, test_item_idx, n_negatives)
        rank = self._ranks(np.array([user_idx]), np.array([test_item_idx]), [negs])
        m = metrics_from_rank(rank, k_values)
        return {k: {n: float(v[0]) for n, v in m[k].items()} for k in k_values}

    def _sample_negatives(self, user_idx: int, test_item_idx: int, n_negatives: int) -> np.ndarray:
        """The reference's sampler (evaluate.py:159-170): one row of _sample_negatives_rows."""
        return self._sample_negatives_rows([user_idx], [test_item_idx], n_negatives)[0]

    def _sample_negatives_rows(self, users, tests, n_negatives: int, arrays: bool = False):
        """The reference's per-row np.random.choice(available, n, replace=False) over all rows in one native
        call (hvae_negatives_legacy): the same draws from numpy's global stream, in row order, which it leaves
        where the per-row calls would. A list of per-row arrays, or with arrays=True (negatives [R, n], counts [R])
        for _ranks."""
        im = self.interaction_matrix
        if getattr(self, "_neg_csr", None) is None or self._neg_csr[0] is not im:
            im = im.tocsr()
            self._neg_csr = (self.interaction_matrix, np.ascontiguousarray(im.indptr, dtype=np.int64),
                             np.ascontiguousarray(im.indices, dtype=np.int32))
        _, indptr, indices = self._neg_csr
        return ops.negatives_legacy(indptr, indices, self.n_items, users, tests, n_negatives, arrays=arrays)

    @staticmethod
    def _candidates(tests: np.ndarray, negatives):
        """[test] + negatives per row as one int32 matrix (cand [R, C], pad [R]: rows padded with their test item
        past their count, cnt [R]). negatives: a list of per-row arrays, or the (negatives [R, n], counts [R])
        block of _sample_negatives_rows(arrays=True), which needs no per-row loop."""
        R = len(tests)
        if isinstance(negatives, tuple):
            neg, cnt = negatives
            cnt = np.asarray(cnt, np.int64)
            C = 1 + (int(cnt.max()) if R else 0)
            cand = np.empty((R, C), np.int32)
            cand[:, 0] = tests
            cand[:, 1:] = neg[:, :C - 1]
            pad = cnt < C - 1
            if pad.any():  # fewer available items than requested: pad with the test item (never outranks)
                fill = np.arange(1, C)[None, :] > cnt[:, None]
                cand[:, 1:] = np.where(fill, np.asarray(tests, np.int32)[:, None], cand[:, 1:])
            return cand, pad, cnt
        cnt = np.array([len(n) for n in negatives], np.int64)
        C = 1 + (int(cnt.max()) if R else 0)
        cand = np.empty((R, C), np.int32)
        pad = np.zeros(R, bool)
        for r, (t, n) in enumerate(zip(tests, negatives)):
            cand[r, 0] = t
            cand[r, 1:1 + len(n)] = n
            if len(n) < C - 1:
                cand[r, 1 + len(n):] = t
                pad[r] = True
        return cand, pad, cnt

    def _ranks(self, users: np.ndarray, tests: np.ndarray, negatives) -> np.ndarray:
        """0-based rank of the test item among [test] + negatives, per row (batched on the device); negatives as
        _candidates takes them."""
        R = len(users)
        cand, pad, cnt = self._candidates(tests, negatives)
        out = np.empty(R, np.int64)
        with torch.no_grad():
            for s in range(0, R, self.batch_size):
                e = min(R, s + self.batch_size)
                u = self._user_vectors(users[s:e])
                cd = torch.as_tensor(cand[s:e], device=self.device)
                sc = ops.score_candidates(u, torch.arange(e - s, dtype=torch.int32, device=self.device), self._E, cd)
                if pad[s:e].any():
                    scn = sc.cpu().numpy()
                    for r in np.nonzero(pad[s:e])[0]:
                        n = int(cnt[s + r])
                        row = scn[r, : 1 + n]
                        out[s + r] = int((row[1:] > row[0]).sum() + (row[1:] == row[0]).sum())
                    rk = ops.rank_first(sc).cpu().numpy()
                    for r in range(e - s):
                        if not pad[s + r]:
                            out[s + r] = rk[r]
                else:
                    out[s:e] = ops.rank_first(sc).cpu().numpy()
        return out

    def evaluate_dataset_with_negatives(self, test_df: pd.DataFrame, n_negatives: int = 99,
                                        k_values: list[int] | None = None) -> dict[int, dict[str, float]]:
        """99-negative protocol over every known (user, item) test row (reference: evaluate.py:187-215)."""
        k_values = k_values or [5, 10, 20]
        logger.info(f"Evaluating with negative sampling ({n_negatives} negatives)...")
        if self.group is not None:  # every rank draws every row's negatives from the same stream
            np.random.seed(broadcast_seed(self.group, self.device))
        users, tests = [], []
        for user_id, item_id in zip(test_df["user_id"].tolist(), test_df["asin"].tolist()):
            if user_id not in self.user_to_idx or item_id not in self.item_to_idx:
                continue
            users.append(self.user_to_idx[user_id])
            tests.append(self.item_to_idx[item_id])
        negs = self._sample_negatives_rows(users, tests, n_negatives, arrays=True)
        all_metrics = {k: {"recall": [], "ndcg": [], "hit_ratio": []} for k in k_values}
        sl = self._shard(len(users))
        if len(users[sl]):
            rank = self._ranks(np.array(users[sl]), np.array(tests[sl]), (negs[0][sl], negs[1][sl]))
            m = metrics_from_rank(rank, k_values)
            for k in k_values:
                for name in ("recall", "ndcg", "hit_ratio"):
                    all_metrics[k][name] = list(m[k][name])
        logger.info(f"Evaluated {len(users)} users")
        return _aggregate_metrics(all_metrics, k_values, self.group, self.device)

    def _shard(self, n: int) -> slice:
        """This rank's rows of a dataset protocol (all rows without a process group)."""
        if self.group is None:
            return slice(0, n)
        import torch.distributed as dist
        return slice(dist.get_rank(self.group), n, dist.get_world_size(self.group))

    def evaluate_user(self, user_id: str, test_items: list[str], k_values: list[int] | None = None):
        k_values = k_values or [5, 10, 20]
        if user_id not in self.user_to_idx:
            return {}
        test_indices = np.array([self.item_to_idx[i] for i in test_items if i in self.item_to_idx])
        if len(test_indices) == 0:
            return {}
        recommended, _ = self.get_user_recommendations(self.user_to_idx[user_id], top_k=max(k_values))
        return {k: {"recall": recall_at_k(recommended, test_indices, k), "ndcg": ndcg_at_k(recommended, test_indices, k),
                    "hit_ratio": hit_ratio_at_k(recommended, test_indices, k)} for k in k_values}

    def evaluate_dataset(self, test_df: pd.DataFrame, k_values: list[int] | None = None):
        """Full-ranking protocol (reference: evaluate.py:243-265), batched top-K on the device."""
        k_values = k_values or [5, 10, 20]
        logger.info("Evaluating with full ranking...")
        test_by_user = test_df.groupby("user_id")["asin"].apply(list).to_dict()
        users, rels = [], []
        for user_id, items in test_by_user.items():
            if user_id not in self.user_to_idx:
                continue
            rel = np.array([self.item_to_idx[i] for i in items if i in self.item_to_idx])
            if len(rel) == 0:
                continue
            users.append(self.user_to_idx[user_id])
            rels.append(rel)
        all_metrics = {k: {"recall": [], "ndcg": [], "hit_ratio": []} for k in k_values}
        K = max(k_values)
        sl = self._shard(len(users))
        users, rels = users[sl], rels[sl]
        for s in range(0, len(users), self.batch_size):
            idx, _ = self._topk(np.array(users[s:s + self.batch_size]), K, True)
            for r, rel in enumerate(rels[s:s + self.batch_size]):
                for k in k_values:
                    all_metrics[k]["recall"].append(recall_at_k(idx[r], rel, k))
                    all_metrics[k]["ndcg"].append(ndcg_at_k(idx[r], rel, k))
                    all_metrics[k]["hit_ratio"].append(hit_ratio_at_k(idx[r], rel, k))
        logger.info(f"Evaluated {len(users)} users")
        return _aggregate_metrics(all_metrics, k_values, self.group, self.device)


# =============================================================================
# Main Functions (reference: evaluate.py:273-370)
# =============================================================================


def load_model_from_checkpoint(checkpoint_path: str, item_embeddings: np.ndarray, device: torch.device) -> HybridVAE:
    logger.info(f"Loading model from {checkpoint_path}")
    # tensors + plain containers only: our own checkpoints (and the reference's) load without unpickling code
    checkpoint = torch.load(checkpoint_path, map_location=device, weights_only=True)
    cfg = checkpoint["model_config"]
    model = create_hybrid_vae(n_items=cfg["n_items"], item_embeddings=item_embeddings, latent_dim=cfg["latent_dim"],
                              hidden_dims=cfg.get("hidden_dims"), dropout=cfg.get("dropout", 0.5),
                              beta=cfg.get("beta", 0.2))
    model.load_state_dict(checkpoint["model_state_dict"])
    logger.info(f"Loaded model from epoch {checkpoint['epoch']}")
    return model


def evaluate_recommendation_model(model_path: str, data_dir: str, embeddings_path: str,
                                  k_values: list[int] | None = None, device: str | None = None,
                                  n_negatives: int | None = None) -> dict:
    k_values = k_values or [5, 10, 20]
    group = init_from_env() if (device is None or str(device).startswith("cuda")) else None  # torchrun: shard rows
    device = _get_device(device)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    full_matrix, train_df, val_df, mappings = load_training_data(data_dir)
    user_to_idx, item_to_idx = mappings["user_to_idx"], mappings["item_to_idx"]
    input_matrix = _build_input_matrix(train_df, val_df, user_to_idx, item_to_idx, full_matrix.shape)
    test_df = pd.read_csv(Path(data_dir) / "test.csv")
    embeddings, _, _ = load_embeddings(embeddings_path)
    model = load_model_from_checkpoint(model_path, embeddings, device)
    evaluator = RecommendationEvaluator(model, input_matrix, user_to_idx, item_to_idx, device, process_group=group)
    if n_negatives is not None:
        protocol = f"NEGATIVE SAMPLING ({n_negatives} negatives)"
        results = evaluator.evaluate_dataset_with_negatives(test_df, n_negatives, k_values)
    else:
        protocol = "FULL RANKING (all items)"
        results = evaluator.evaluate_dataset(test_df, k_values)
    if is_main(group):
        logger.info(f"\n{'=' * 70}\nHYBRID VAE EVALUATION RESULTS\nProtocol: {protocol}\n{'=' * 70}")
        print(f"\n{'-' * 70}\n{'K':<5} | {'Recall':>12} | {'NDCG':>12} | {'Hit Ratio':>12}\n{'-' * 70}")
        for k in k_values:
            m = results[k]
            print(f"@{k:<4} | {m['recall']:>12.4f} | {m['ndcg']:>12.4f} | {m['hit_ratio']:>12.4f}")
        print("-" * 70)
    return results


def main() -> None:
    parser = argparse.ArgumentParser(description="Evaluate recommendation model (MI355X)")
    parser.add_argument("--model", default=config.MODEL_FILE)
    parser.add_argument("--data", default=str(config.DATA_DIR))
    parser.add_argument("--embeddings", default=config.EMBEDDINGS_FILE)
    parser.add_argument("--k-values", type=int, nargs="+", default=[5, 10, 20])
    parser.add_argument("--device", choices=["cuda", "cpu", "mps"])
    parser.add_argument("--output", help="Path to save results (JSON)")
    parser.add_argument("--n-negatives", type=int, default=99, help="Negatives count (0 for full ranking)")
    args = parser.parse_args()
    n_negatives = args.n_negatives if args.n_negatives > 0 else None
    results = evaluate_recommendation_model(model_path=args.model, data_dir=args.data, embeddings_path=args.embeddings,
                                            k_values=args.k_values, device=args.device, n_negatives=n_negatives)
    if args.output and is_main(init_from_env()):
        with open(args.output, "w") as f:
            json.dump(results, f, indent=2)
        logger.info(f"Results saved to {args.output}")


if __name__ == "__main__":
    main()
