"""G7: NDCG@K statistical fixture from the reference's own `make train-best` / `make evaluate` path.

Run in the build container (where /root/reference exists), in the background (~7 min per seed on 6 threads):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_ndcg_fixture.py [n_seeds] [first_seed] [threads]
Seeds already in ndcg_planted.json are kept: a later run with first_seed > 0 appends its seeds, so the
fixture grows one seed at a time (each seed's run is written as soon as it finishes).

The All_Beauty data cannot be fetched here, so the offline stand-in is an
All_Beauty-shaped planted-cluster dataset (gen.synth_planted: 22,363 users x 12,101 items,
d = 384, leave-one-out splits) written in the reference's on-disk layout. For each seed the
reference's train_hybrid_vae (src/ml/train.py:199-332, best config latent 128, hidden [512],
dropout 0.3, beta 0.2, lr 1e-3, batch 64, 20 epochs) trains on CPU, then its
evaluate_recommendation_model (src/ml/evaluate.py:294-340) scores best_model.pth with the
1 + 99 negative protocol, numpy seeded with neg_seed right before, so the negatives are the
same in every run and in ours. Only the metrics are stored (tests/golden/ndcg_planted.json).
"""
from __future__ import annotations

import json
import random
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
from gen import PLANTED_CONFIG, digest, synth_planted, write_planted_artifacts  # noqa: E402
from make_golden import import_reference  # noqa: E402


def main():
    import torch
    n_seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    torch.set_num_threads(int(sys.argv[3]) if len(sys.argv) > 3 else 6)
    _, train_m, eval_m = import_reference()
    c = PLANTED_CONFIG
    path = HERE / "ndcg_planted.json"
    old = json.loads(path.read_text()) if (first > 0 and path.exists()) else {"runs": []}
    runs = [r for r in old["runs"] if r["seed"] < first]
    tr, va, te, E, _, _ = synth_planted(**c)
    data_digest = digest(tr["user_id"].str[1:].astype(np.int64).values, tr["asin"].str[1:].astype(np.int64).values,
                         va["asin"].str[1:].astype(np.int64).values, te["asin"].str[1:].astype(np.int64).values, E)
    assert old.get("data_digest", data_digest) == data_digest, "planted dataset changed since the kept seeds"

    def save():
        nd = np.array([r["metrics"]["10"]["ndcg"] for r in runs])
        fix = {"config": c, "torch": torch.__version__, "runs": runs,
               "ndcg10_mean": float(nd.mean()), "ndcg10_std": float(nd.std(ddof=1)) if len(nd) > 1 else 0.0,
               "data_digest": data_digest}
        path.write_text(json.dumps(fix, indent=1))
        return fix

    with tempfile.TemporaryDirectory() as td:
        data, emb = write_planted_artifacts(td)
        for s in range(first, first + n_seeds):
            out = Path(td) / f"models_{s}"
            torch.manual_seed(s)
            np.random.seed(s)
            random.seed(s)
            t0 = time.time()
            train_m.train_hybrid_vae(str(data), str(emb), str(out), latent_dim=c["latent"], hidden_dims=c["hidden"],
                                     batch_size=c["batch"], epochs=c["epochs"], learning_rate=c["lr"],
                                     beta=c["beta"], dropout=c["dropout"], device="cpu", patience=20)
            t1 = time.time()
            np.random.seed(c["neg_seed"])
            res = eval_m.evaluate_recommendation_model(str(out / "best_model.pth"), str(data), str(emb),
                                                       k_values=[5, 10, 20], device="cpu", n_negatives=99)
            hist = json.loads((out / "training_history.json").read_text())
            runs.append({"seed": s, "train_s": round(t1 - t0, 1), "eval_s": round(time.time() - t1, 1),
                         "metrics": {str(k): v for k, v in res.items()},
                         "val_losses": hist["val_losses"], "train_losses": hist["train_losses"]})
            print(json.dumps(runs[-1]), flush=True)
            fix = save()
    print("ndcg@10", fix["ndcg10_mean"], "+-", fix["ndcg10_std"], "over", len(runs), "seeds")


if __name__ == "__main__":
    main()
