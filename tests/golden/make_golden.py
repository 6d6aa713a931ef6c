"""Generate the golden vectors that pin the CPU oracle to the reference.

Run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own src/ml modules (two absent third-party imports
are stubbed: python-dotenv's load_dotenv -> no-op, sentence_transformers'
SentenceTransformer -> placeholder; neither is on the path exercised here) and
records, for fixed synthetic inputs (tests/golden/gen.py):
  G1 eval forward   (HybridVAE.eval(): mu, logvar, projection(mu), scores, loss terms, top-10)
  G2 train steps    (VAETrainer.train_epoch on one batch, dropout masks and eps injected;
                     pre-clip grads, clip norm, params + Adam moments after 2 steps)
  G3 metric KATs    (recall_at_k, ndcg_at_k, hit_ratio_at_k)
  G4 eval protocol  (evaluate_user_with_negatives / evaluate_dataset_with_negatives with
                     fixed negatives; get_user_recommendations top-20)
  G5 CSR semantics  (_build_matrix / _build_input_matrix: positives filter, duplicate sums)
  G6 API contract   (state_dict keys / shapes / reference init checksums)
Only inputs -> outputs are stored; no reference source is copied.
"""
from __future__ import annotations

import json
import os
import sys
import types
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
from gen import EVAL_CONFIG, TRAIN_CONFIGS, digest, synth_csr, synth_embeddings, synth_eps, synth_masks  # noqa: E402

REF = Path(os.environ.get("HVAE_REFERENCE", "/root/reference"))


def import_reference():
    d = types.ModuleType("dotenv")
    d.load_dotenv = lambda *a, **k: None
    sys.modules.setdefault("dotenv", d)
    st = types.ModuleType("sentence_transformers")
    st.SentenceTransformer = object
    sys.modules.setdefault("sentence_transformers", st)
    sys.path[:0] = [str(REF), str(REF / "src")]
    import src.ml.evaluate as ev
    import src.ml.model as model
    import src.ml.train as train
    return model, train, ev


def main():
    import torch
    model_m, train_m, eval_m = import_reference()
    out: dict[str, np.ndarray] = {}
    meta: dict = {"reference": str(REF), "torch": torch.__version__, "numpy": np.__version__}

    # ------------------------------------------------------------ G1 ------
    c = EVAL_CONFIG
    X = synth_csr(c["n_users"], c["n_items"], seed=100)
    E = synth_embeddings(c["n_items"], c["d"], seed=101)
    torch.manual_seed(c["seed"])
    m = model_m.HybridVAE(c["n_items"], E, latent_dim=c["latent"], hidden_dims=c["hidden"], dropout=0.3, beta=c["beta"])
    m.eval()
    x = torch.as_tensor(X.toarray(), dtype=torch.float32)
    with torch.no_grad():
        mu, lv = m.encode(x)
        u = m.projection_layer(mu)
        scores = m.decode(mu)
        rc, lv2 = m(x)[0], None
        total, recon, kl = model_m.vae_loss_function(rc, x, mu, lv, c["beta"])
    s = scores.numpy()
    out["g1_mu"] = mu.numpy()
    out["g1_logvar"] = lv.numpy()
    out["g1_u"] = u.numpy()
    out["g1_scores"] = s
    out["g1_loss"] = np.array([total.item(), recon.item(), kl.item()], np.float64)
    out["g1_top10"] = np.stack([np.argsort(r, kind="stable")[::-1][:10] for r in s]).astype(np.int64)
    meta["g1_inputs"] = digest(X.indptr, X.indices, X.data, E)
    sd = {k: v.detach().numpy() for k, v in m.state_dict().items()}
    meta["g1_state_checksum"] = {k: [float(np.float64(v).sum()), float((np.float64(v) ** 2).sum())] for k, v in sd.items()}
    out["g1_w1_head"] = sd["encoder.0.weight"][:4, :16].copy()
    out["g1_proj_head"] = sd["projection_layer.3.weight"][:4, :16].copy()

    # ------------------------------------------------------------ G4 ------
    ev_model = m
    n_users = c["n_users"]
    user_to_idx = {f"u{i}": i for i in range(n_users)}
    item_to_idx = {f"i{j}": j for j in range(c["n_items"])}
    rng = np.random.Generator(np.random.PCG64(102))
    test_rows = []
    for i in range(n_users):
        seen = set(X[i].indices.tolist())
        cand = [j for j in range(c["n_items"]) if j not in seen]
        test_rows.append((i, int(rng.choice(cand))))
    import pandas as pd
    test_df = pd.DataFrame({"user_id": [f"u{i}" for i, _ in test_rows], "asin": [f"i{j}" for _, j in test_rows]})
    # fixed negatives: the evaluator's np.random.choice(available, 99, replace=False) is
    # replaced by a deterministic draw recorded here
    negs = []
    for i, t in test_rows:
        seen = set(X[i].indices.tolist())
        avail = np.array([j for j in range(c["n_items"]) if j not in seen and j != t])
        negs.append(rng.choice(avail, 99, replace=False))
    negs = np.stack(negs).astype(np.int64)
    it = iter(list(negs))
    orig_choice = np.random.choice
    np.random.choice = lambda a, n, replace=True: next(it)
    try:
        evaluator = eval_m.RecommendationEvaluator(ev_model, X, user_to_idx, item_to_idx, torch.device("cpu"))
        res = evaluator.evaluate_dataset_with_negatives(test_df, 99, [5, 10, 20])
    finally:
        np.random.choice = orig_choice
    out["g4_test_items"] = np.array([t for _, t in test_rows], np.int64)
    out["g4_negatives"] = negs
    out["g4_metrics"] = np.array([[res[k]["recall"], res[k]["ndcg"], res[k]["hit_ratio"]] for k in (5, 10, 20)])
    recs = [evaluator.get_user_recommendations(i, top_k=20) for i in range(8)]
    out["g4_full_top20"] = np.stack([r[0] for r in recs]).astype(np.int64)
    out["g4_full_top20_scores"] = np.stack([r[1] for r in recs]).astype(np.float32)

    # ------------------------------------------------------------ G2 ------
    for name, c in TRAIN_CONFIGS.items():
        X = synth_csr(c["n_users"], c["n_items"], lam=c.get("lam", 3.0), seed=200 + c["seed"])
        E = synth_embeddings(c["n_items"], c["d"], seed=300 + c["seed"])
        torch.manual_seed(c["seed"])
        mdl = model_m.HybridVAE(c["n_items"], E, latent_dim=c["latent"], hidden_dims=c["hidden"],
                                dropout=c["dropout"], beta=c["beta"])
        trainer = train_m.VAETrainer(mdl, torch.device("cpu"), lr=c["lr"], weight_decay=c.get("wd", 0.0))
        x = torch.as_tensor(X.toarray(), dtype=torch.float32)
        B = c["n_users"]
        has_proj = c["latent"] != c["d"]
        rec = {"norm": [], "loss": []}
        for step in (1, 2):
            enc_m = synth_masks([(B, h) for h in c["hidden"]], c["dropout"], seed=400 + 10 * step + c["seed"])
            proj_m = synth_masks([(B, c["d"])], c["dropout"], seed=500 + 10 * step + c["seed"])[0]
            eps = synth_eps((B, c["latent"]), seed=600 + 10 * step + c["seed"])
            for k, mk in enumerate(enc_m):
                out[f"g2{name}_s{step}_encmask{k}"] = mk
            if has_proj:
                out[f"g2{name}_s{step}_projmask"] = proj_m
            out[f"g2{name}_s{step}_eps"] = eps
            # inject: Dropout modules -> fixed multipliers, randn_like -> eps
            masks = iter(enc_m)
            for k in range(len(c["hidden"])):
                mk = torch.as_tensor(next(masks))
                mdl.encoder[4 * k + 3] = _Mask(mk)
            if has_proj:
                mdl.projection_layer[2] = _Mask(torch.as_tensor(proj_m))
            orig_rl = torch.randn_like
            orig_clip = torch.nn.utils.clip_grad_norm_
            captured = {}

            def clip_spy(params, max_norm, *a, **k):
                params = list(params)
                captured["grads"] = {n: p.grad.detach().clone() for n, p in mdl.named_parameters()}
                r = orig_clip(params, max_norm, *a, **k)
                captured["norm"] = float(r)
                return r

            torch.randn_like = lambda t, *a, **k: torch.as_tensor(eps).to(t.dtype)
            torch.nn.utils.clip_grad_norm_ = clip_spy
            try:
                metrics = trainer.train_epoch([x])
            finally:
                torch.randn_like = orig_rl
                torch.nn.utils.clip_grad_norm_ = orig_clip
            rec["norm"].append(captured["norm"])
            rec["loss"].append([metrics["total_loss"], metrics["recon_loss"], metrics["kl_loss"]])
            if step == 1:
                for n, g in captured["grads"].items():
                    out[f"g2{name}_s1_grad_{n}"] = g.numpy()
        for n, p in mdl.named_parameters():
            out[f"g2{name}_s2_param_{n}"] = p.detach().numpy()
            st = trainer.optimizer.state[p]
            out[f"g2{name}_s2_m_{n}"] = st["exp_avg"].numpy()
            out[f"g2{name}_s2_v_{n}"] = st["exp_avg_sq"].numpy()
        out[f"g2{name}_norm"] = np.array(rec["norm"], np.float64)
        out[f"g2{name}_loss"] = np.array(rec["loss"], np.float64)
        meta[f"g2{name}_inputs"] = digest(X.indptr, X.indices, X.data, E)

    # ------------------------------------------------------------ G3 ------
    rng = np.random.Generator(np.random.PCG64(700))
    kat = []
    for trial in range(40):
        n_rec = int(rng.integers(0, 30))
        recd = rng.choice(50, size=n_rec, replace=False)
        n_rel = int(rng.integers(0, 6))
        rel = rng.choice(50, size=n_rel, replace=False)
        for k in (1, 5, 10, 20):
            kat.append((trial, k, eval_m.recall_at_k(recd, rel, k), eval_m.ndcg_at_k(recd, rel, k),
                        eval_m.hit_ratio_at_k(recd, rel, k)))
        out[f"g3_rec_{trial}"] = recd.astype(np.int64)
        out[f"g3_rel_{trial}"] = rel.astype(np.int64)
    out["g3_kat"] = np.array(kat, np.float64)

    # ------------------------------------------------------------ G5 ------
    df = pd.DataFrame({
        "user_id": ["a", "a", "b", "b", "b", "c", "c", "a", "d"],
        "asin": ["x", "x", "y", "z", "y", "x", "w", "w", "z"],
        "binary_rating": [1, 1, 1, 0, 1, 0, 1, 1, 0],
    })
    val = pd.DataFrame({"user_id": ["a", "c", "d"], "asin": ["y", "x", "x"], "binary_rating": [1, 1, 0]})
    u2i = {u: i for i, u in enumerate("abcd")}
    i2i = {a: i for i, a in enumerate("wxyz")}
    M = train_m._build_matrix(df, u2i, i2i, (4, 4))
    Mi = eval_m._build_input_matrix(df, val, u2i, i2i, (4, 4))
    out["g5_train_dense"] = M.toarray()
    out["g5_input_dense"] = Mi.toarray()
    out["g5_users_in_train"] = np.array(train_m.get_user_indices_from_df(df, u2i), np.int64)

    # ------------------------------------------------------------ G6 ------
    torch.manual_seed(0)
    big = model_m.HybridVAE(50, synth_embeddings(50, 384, seed=5), latent_dim=128, hidden_dims=[512, 256])
    meta["g6_state_dict"] = {k: list(v.shape) for k, v in big.state_dict().items()}
    meta["g6_param_order"] = [n for n, _ in big.named_parameters()]
    meta["g6_adam_defaults"] = {k: (list(v) if isinstance(v, tuple) else v)
                                for k, v in torch.optim.Adam(big.parameters()).defaults.items()
                                if isinstance(v, (int, float, bool, tuple)) or v is None}

    np.savez_compressed(HERE / "golden.npz", **out)
    (HERE / "golden_meta.json").write_text(json.dumps(meta, indent=1, sort_keys=True))
    size = (HERE / "golden.npz").stat().st_size
    print(f"wrote {len(out)} arrays, {size / 1e6:.2f} MB")


class _Mask:
    """Stand-in for nn.Dropout: multiply by a fixed multiplier tensor in train mode."""

    def __new__(cls, mult):
        import torch

        class Mask(torch.nn.Module):
            def __init__(self, mult):
                super().__init__()
                self.mult = mult

            def forward(self, h):
                return h * self.mult if self.training else h

        return Mask(mult)


if __name__ == "__main__":
    main()
