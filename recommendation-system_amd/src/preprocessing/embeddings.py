"""Item-embedding file format consumed by the hot path.

Mirrors load_embeddings / the save format of src/preprocessing/embeddings.py
(:93-158): ``<name>.npy`` (float32 [N, d], L2-normalised rows, items sorted by
asin) plus ``<name>_mappings.pkl`` ({item_to_idx, idx_to_item, embedding_dim,
model_name, n_items}). SBERT generation itself (:27-91) needs a model fetched
by name from the HF hub and is out of scope here.
"""
from __future__ import annotations

import logging
import pickle
from pathlib import Path

import numpy as np

logger = logging.getLogger(__name__)


def load_embeddings(embeddings_path, mappings_path=None):
    """(embeddings, item_to_idx | None, idx_to_item | None), as embeddings.py:134-158."""
    embeddings_path = Path(embeddings_path)
    embeddings = np.load(embeddings_path)
    item_to_idx, idx_to_item = None, None
    if mappings_path is None:
        mappings_path = embeddings_path.with_name(f"{embeddings_path.stem}_mappings.pkl")
    if Path(mappings_path).exists():
        with open(mappings_path, "rb") as f:
            mappings = pickle.load(f)  # the project's own artifact (written by save_embeddings)
        item_to_idx = mappings.get("item_to_idx")
        idx_to_item = mappings.get("idx_to_item")
    logger.info("Loaded embeddings %s", embeddings.shape)
    return embeddings, item_to_idx, idx_to_item


def save_embeddings(embeddings: np.ndarray, item_to_idx: dict, idx_to_item: dict, output_path,
                    model_name: str = "all-MiniLM-L6-v2") -> None:
    """Write the three files of ItemEmbeddingGenerator.save_embeddings (embeddings.py:93-131)."""
    out = Path(output_path)
    out.parent.mkdir(parents=True, exist_ok=True)
    np.save(out, embeddings)
    with open(out.with_name(f"{out.stem}_mappings.pkl"), "wb") as f:
        pickle.dump({"item_to_idx": item_to_idx, "idx_to_item": idx_to_item,
                     "embedding_dim": int(embeddings.shape[1]), "model_name": model_name,
                     "n_items": len(item_to_idx)}, f)
    out.with_name(f"{out.stem}_metadata.txt").write_text(
        f"Model: {model_name}\nDimension: {embeddings.shape[1]}\nItems: {len(item_to_idx)}\n"
        f"Shape: {embeddings.shape}\nDevice: n/a\n")
