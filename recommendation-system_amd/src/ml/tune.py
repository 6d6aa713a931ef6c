"""Hyperparameter grid search for HybridVAE on MI355X (drop-in for the reference's src/ml/tune.py).

Same search space, flags, outputs (models/grid_search_results.json with the "best_config" that
`make train-best` reads) and selection rule (best NDCG@10 on the validation split, 1 + 99
negatives) as the reference (tune.py:35-360). Every configuration trains through the fused HIP
train step (hvae.executor.FusedTrainer via VAETrainer: one graph replay per batch, the annealed
beta computed on the device by the replayed step itself) and is scored by the device evaluator's batched candidate ranking, instead of
the reference's per-row densifying loader and per-user Python loop.
"""
from __future__ import annotations

import argparse
import itertools
import json
import logging
from datetime import datetime
from pathlib import Path
from typing import Any

import numpy as np
import pandas as pd
import torch
from scipy.sparse import csr_matrix
from torch.utils.data import DataLoader

from src.config import config
from src.ml.evaluate import RecommendationEvaluator, metrics_from_rank
from src.ml.model import create_hybrid_vae
from src.ml.train import UserInteractionDataset, VAETrainer, get_user_indices_from_df, load_training_data
from src.preprocessing.embeddings import load_embeddings

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger(__name__)

# reference: tune.py:35-41
DEFAULT_SEARCH_SPACE = {
    "latent_dim": [32, 64, 128],
    "hidden_dims": [[256], [512], [256, 128]],
    "dropout": [0.3, 0.5],
    "beta": [0.1, 0.2, 0.3],
    "learning_rate": [1e-3, 5e-4],
}


def _get_device(device: str | None = None) -> torch.device:
    if device:
        dev = torch.device(device)
        if dev.type != "cuda":  # the reference's cpu / mps choices parse, then fail here, before any data loads
            raise RuntimeError(f"device {device!r}: the MI355X HybridVAE path runs on a HIP device only; "
                               "there is no CPU fallback.")
        return dev
    if torch.cuda.is_available():
        return torch.device("cuda")
    raise RuntimeError("The MI355X HybridVAE path needs a HIP device (torch.cuda on ROCm); none is visible. "
                       "There is no CPU fallback.")


def _build_interaction_matrix(df: pd.DataFrame, user_to_idx: dict, item_to_idx: dict, shape: tuple) -> csr_matrix:
    """Positives with duplicate pairs summed (reference: tune.py:55-60)."""
    positives = df[df["binary_rating"] == 1] if "binary_rating" in df.columns else df
    rows = positives["user_id"].map(user_to_idx)
    cols = positives["asin"].map(item_to_idx)
    return csr_matrix((np.ones(len(positives)), (rows, cols)), shape=shape)


def train_single_config(model, train_loader: DataLoader, val_loader: DataLoader, device: torch.device,
                        learning_rate: float, epochs: int = 10, patience: int = 3) -> tuple[float, int]:
    """Train with Adam + clip 5.0, early-stop on the validation loss; (best val loss, best epoch).

    Reference: tune.py:63-116 (the epoch's val loss is the mean of per-batch losses, as there).
    """
    trainer = VAETrainer(model, device, lr=learning_rate)
    best_val_loss, best_epoch, patience_counter = float("inf"), 0, 0
    for epoch in range(epochs):
        trainer.train_epoch(train_loader)
        val_loss = trainer.validate(val_loader)["total_loss"]
        if val_loss < best_val_loss:
            best_val_loss, best_epoch, patience_counter = val_loss, epoch + 1, 0
        else:
            patience_counter += 1
            if patience_counter >= patience:
                break
    return best_val_loss, best_epoch


def evaluate_config_on_val(model, train_matrix: csr_matrix, val_df: pd.DataFrame, user_to_idx: dict,
                           item_to_idx: dict, device: torch.device, n_negatives: int = 99,
                           k_values: list[int] | None = None) -> dict[str, float]:
    """Validation NDCG / recall / HR with 1 + n_negatives candidates per val row (reference: tune.py:119-180).

    The model's input rows are the TRAIN positives (not train + val, unlike evaluate.py). Negatives
    are drawn with the reference's sampler, row by row in val_df order, so a seeded numpy RNG yields
    the same candidate lists; the candidates are scored and ranked on the device in user batches.
    """
    k_values = k_values or [10]
    ev = RecommendationEvaluator(model, train_matrix, user_to_idx, item_to_idx, device)
    users, tests = [], []
    for user_id, item_id in zip(val_df["user_id"].tolist(), val_df["asin"].tolist()):
        if user_id not in user_to_idx or item_id not in item_to_idx:
            continue
        users.append(user_to_idx[user_id])
        tests.append(item_to_idx[item_id])
    negs = ev._sample_negatives_rows(users, tests, n_negatives, arrays=True)
    if not users:
        return {f"{m}@{k}": 0.0 for k in k_values for m in ("recall", "ndcg", "hit_ratio")}
    rank = ev._ranks(np.array(users), np.array(tests), negs)
    m = metrics_from_rank(rank, k_values)
    return {f"{name}@{k}": float(np.mean(m[k][name])) for k in k_values for name in ("recall", "ndcg", "hit_ratio")}


class _GridData:
    """What every configuration of one grid search reads: the split matrices, loaders and the embeddings."""

    def __init__(self, data_dir: str, embeddings_path: str, batch_size: int, device: str | None):
        self.dev = _get_device(device)
        full_matrix, train_df, self.val_df, mappings = load_training_data(data_dir)
        self.user_to_idx, self.item_to_idx = mappings["user_to_idx"], mappings["item_to_idx"]
        self.n_items = full_matrix.shape[1]
        self.train_matrix = _build_interaction_matrix(train_df, self.user_to_idx, self.item_to_idx, full_matrix.shape)
        val_matrix = _build_interaction_matrix(self.val_df, self.user_to_idx, self.item_to_idx, full_matrix.shape)
        emb_path = Path(embeddings_path)
        self.embeddings, _, _ = load_embeddings(embeddings_path,
                                                str(emb_path.with_name(f"{emb_path.stem}_mappings.pkl")))
        self.train_loader = DataLoader(
            UserInteractionDataset(self.train_matrix, get_user_indices_from_df(train_df, self.user_to_idx)),
            batch_size=batch_size, shuffle=True, num_workers=0)
        self.val_loader = DataLoader(
            UserInteractionDataset(val_matrix, get_user_indices_from_df(self.val_df, self.user_to_idx)),
            batch_size=batch_size, shuffle=False, num_workers=0)


def _one_config(g: _GridData, cfg: dict, use_annealing: bool, epochs: int, patience: int,
                seed: int | None) -> dict[str, Any]:
    """Train and score one grid point (reference: tune.py:240-279); failures are recorded, not raised."""
    try:
        if seed is not None:  # concurrent grids: every configuration from its own seed, wherever it runs
            torch.manual_seed(seed)
            np.random.seed(seed % 2 ** 32)
        model = create_hybrid_vae(n_items=g.n_items, item_embeddings=g.embeddings,
                                  latent_dim=cfg.get("latent_dim", 64), hidden_dims=cfg.get("hidden_dims", [256]),
                                  dropout=cfg.get("dropout", 0.5), beta=cfg.get("beta", 0.2),
                                  use_annealing=use_annealing, anneal_steps=len(g.train_loader) * epochs // 2)
        val_loss, best_epoch = train_single_config(model, g.train_loader, g.val_loader, g.dev,
                                                   learning_rate=cfg.get("learning_rate", 1e-3),
                                                   epochs=epochs, patience=patience)
        metrics = evaluate_config_on_val(model, g.train_matrix, g.val_df, g.user_to_idx, g.item_to_idx, g.dev,
                                         n_negatives=99, k_values=[10])
        return {"config": cfg, "val_loss": val_loss, "best_epoch": best_epoch, **metrics}
    except Exception as e:  # the reference records the failure and moves on (tune.py:277-279)
        logger.error(f"  Failed: {e}")
        return {"config": cfg, "error": str(e)}
    finally:
        torch.cuda.empty_cache()


_WORKER: dict[str, Any] = {}


def _worker_init(data_dir: str, embeddings_path: str, batch_size: int, device: str | None) -> None:
    _WORKER["grid"] = _GridData(data_dir, embeddings_path, batch_size, device)


def _worker_run(task: tuple) -> tuple[int, dict[str, Any]]:
    i, cfg, use_annealing, epochs, patience, seed = task
    return i, _one_config(_WORKER["grid"], cfg, use_annealing, epochs, patience, seed)


def run_grid_search(data_dir: str, embeddings_path: str, output_dir: str,
                    search_space: dict[str, list] | None = None, epochs_per_config: int = 10, patience: int = 3,
                    batch_size: int = 512, use_annealing: bool = True, device: str | None = None,
                    concurrent: int = 1, seed: int | None = None) -> dict[str, Any]:
    """Grid search over search_space; writes output_dir/grid_search_results.json (reference: tune.py:183-322).

    concurrent > 1 packs that many configurations onto the GPU at once: one process each (spawned, at most 8), each
    loading the data once and taking grid points as they free up. A configuration's train step at B = 512 leaves
    the GPU mostly idle between its short launches, so concurrent ones overlap. Every configuration then starts
    from its own seed (seed + its index; seed defaults to 0 here) so that its result does not depend on which
    process ran it or when: the same grid with the same seed gives the same results at any concurrency. Results
    and the selection (first best NDCG@10 in grid order) are as in the serial search.
    """
    search_space = search_space or DEFAULT_SEARCH_SPACE
    if concurrent < 1 or concurrent > 8:
        raise ValueError("concurrent must be in 1..8 (processes sharing one GPU)")
    output_path = Path(output_dir)
    output_path.mkdir(parents=True, exist_ok=True)
    param_names = list(search_space.keys())
    all_configs = [dict(zip(param_names, values)) for values in itertools.product(*search_space.values())]
    logger.info(f"Grid search over {len(all_configs)} configurations")
    if concurrent > 1 and seed is None:
        seed = 0
    seeds = [None if seed is None else seed + i for i in range(len(all_configs))]
    if concurrent == 1:
        g = _GridData(data_dir, embeddings_path, batch_size, device)
        logger.info(f"Using device: {g.dev}")
        results = []
        for i, cfg in enumerate(all_configs):
            logger.info(f"\n[{i + 1}/{len(all_configs)}] Testing: {cfg}")
            results.append(_one_config(g, cfg, use_annealing, epochs_per_config, patience, seeds[i]))
            r = results[-1]
            if "error" not in r:
                logger.info(f"  Val Loss: {r['val_loss']:.4f}, NDCG@10: {r['ndcg@10']:.4f}, "
                            f"Recall@10: {r['recall@10']:.4f}")
    else:
        _get_device(device)  # fail before spawning when no HIP device is visible
        import multiprocessing as mp
        tasks = [(i, cfg, use_annealing, epochs_per_config, patience, seeds[i]) for i, cfg in enumerate(all_configs)]
        results = [None] * len(all_configs)
        with mp.get_context("spawn").Pool(concurrent, initializer=_worker_init,
                                          initargs=(data_dir, embeddings_path, batch_size, device)) as pool:
            for i, r in pool.imap_unordered(_worker_run, tasks):
                results[i] = r
                logger.info(f"[{i + 1}/{len(all_configs)}] {r['config']}: "
                            + (f"NDCG@10 {r['ndcg@10']:.4f}" if "error" not in r else f"failed: {r['error']}"))
    best_config, best_metric = None, -float("inf")
    for r in results:
        if "error" not in r and r["ndcg@10"] > best_metric:
            best_metric, best_config = r["ndcg@10"], r["config"]

    valid_results = sorted([r for r in results if "error" not in r], key=lambda x: x["ndcg@10"], reverse=True)
    output_file = output_path / "grid_search_results.json"
    with open(output_file, "w") as f:
        json.dump({"search_space": {k: [str(v) for v in vals] for k, vals in search_space.items()},
                   "best_config": best_config, "best_ndcg@10": best_metric, "all_results": results,
                   "timestamp": datetime.now().isoformat()}, f, indent=2, default=str)
    logger.info(f"\nGrid search complete! Results saved to {output_file}")
    logger.info(f"Best config: {best_config}")
    logger.info(f"Best NDCG@10: {best_metric:.4f}")
    logger.info("\nTop 5 configurations:")
    for i, r in enumerate(valid_results[:5]):
        logger.info(f"  {i + 1}. NDCG@10={r['ndcg@10']:.4f}, Recall@10={r['recall@10']:.4f}, config={r['config']}")
    return {"best_config": best_config, "best_metric": best_metric, "all_results": results}


def main() -> None:
    """CLI of `make tune` (reference: tune.py:325-356)."""
    parser = argparse.ArgumentParser(description="Hyperparameter tuning for Hybrid VAE")
    parser.add_argument("--data", default=str(config.DATA_DIR), help="Data directory")
    parser.add_argument("--embeddings", default=str(config.EMBEDDINGS_FILE), help="Embeddings path")
    parser.add_argument("--output", default=str(config.MODEL_DIR), help="Output directory")
    parser.add_argument("--epochs", type=int, default=10, help="Max epochs per config")
    parser.add_argument("--patience", type=int, default=3, help="Early stopping patience")
    parser.add_argument("--batch-size", type=int, default=512, help="Batch size")
    parser.add_argument("--device", choices=["cuda", "mps", "cpu"],
                        help="Device (reference flag; only a HIP device runs: cpu / mps raise, there is no CPU fallback)")
    parser.add_argument("--latent-dims", type=int, nargs="+", default=[32, 64, 128])
    parser.add_argument("--dropouts", type=float, nargs="+", default=[0.3, 0.5])
    parser.add_argument("--betas", type=float, nargs="+", default=[0.1, 0.2, 0.3])
    parser.add_argument("--learning-rates", type=float, nargs="+", default=[1e-3, 5e-4])
    parser.add_argument("--concurrent", type=int, default=1,
                        help="configurations trained at once on the GPU, one process each (1-8; MI355X addition)")
    parser.add_argument("--seed", type=int, default=None,
                        help="seed configuration i with seed + i (default with --concurrent > 1: 0)")
    args = parser.parse_args()
    run_grid_search(data_dir=args.data, embeddings_path=args.embeddings, output_dir=args.output,
                    search_space={"latent_dim": args.latent_dims, "hidden_dims": [[256], [512], [256, 128]],
                                  "dropout": args.dropouts, "beta": args.betas, "learning_rate": args.learning_rates},
                    epochs_per_config=args.epochs, patience=args.patience, batch_size=args.batch_size,
                    device=args.device, concurrent=args.concurrent, seed=args.seed)


if __name__ == "__main__":
    main()
