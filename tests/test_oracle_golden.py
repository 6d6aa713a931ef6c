"""Pin the CPU oracle (oracle/ref_cpu.py) against golden vectors of the reference.

The golden vectors were produced by importing the reference itself
(tests/golden/make_golden.py); these tests run on CPU everywhere.
"""
import numpy as np
import pandas as pd
import pytest
import torch

from gen import EVAL_CONFIG, TRAIN_CONFIGS, digest, synth_csr, synth_embeddings
from oracle import ref_cpu as R


def _close(a, b, rtol, atol, what):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.max(np.abs(a - b) / (atol + rtol * np.abs(b))) if a.size else 0.0
    assert a.shape == b.shape and err <= 1.0, f"{what}: scaled err {err:.3g}"


def _close_max(a, b, tol, what):
    """max|a - b| <= tol * max|b|: for sums with cancellation (gradients, moments)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(np.max(np.abs(b)), 1e-30)
    err = np.max(np.abs(a - b)) / scale
    assert a.shape == b.shape and err <= tol, f"{what}: max err {err:.3g} x max|ref|"


def test_inputs_are_reproducible(golden_meta):
    c = EVAL_CONFIG
    X = synth_csr(c["n_users"], c["n_items"], seed=100)
    E = synth_embeddings(c["n_items"], c["d"], seed=101)
    assert digest(X.indptr, X.indices, X.data, E) == golden_meta["g1_inputs"]
    for name, c in TRAIN_CONFIGS.items():
        X = synth_csr(c["n_users"], c["n_items"], lam=c.get("lam", 3.0), seed=200 + c["seed"])
        E = synth_embeddings(c["n_items"], c["d"], seed=300 + c["seed"])
        assert digest(X.indptr, X.indices, X.data, E) == golden_meta[f"g2{name}_inputs"]


def test_init_matches_reference(golden, golden_meta):
    c = EVAL_CONFIG
    E = synth_embeddings(c["n_items"], c["d"], seed=101)
    p = R.init_params(c["n_items"], E, c["latent"], c["hidden"], seed=c["seed"])
    for k, (s1, s2) in golden_meta["g1_state_checksum"].items():
        v = p[k].double().numpy()
        assert abs(v.sum() - s1) <= 1e-6 * max(1.0, abs(s1)) + 1e-9, k
        assert abs((v ** 2).sum() - s2) <= 1e-9 * max(1.0, s2), k
    np.testing.assert_array_equal(p["encoder.0.weight"][:4, :16].numpy(), golden["g1_w1_head"])
    np.testing.assert_array_equal(p["projection_layer.3.weight"][:4, :16].numpy(), golden["g1_proj_head"])


def test_eval_forward(golden):
    c = EVAL_CONFIG
    X = synth_csr(c["n_users"], c["n_items"], seed=100)
    E = synth_embeddings(c["n_items"], c["d"], seed=101)
    p = R.init_params(c["n_items"], E, c["latent"], c["hidden"], seed=c["seed"])
    x = torch.as_tensor(X.toarray(), dtype=torch.float32)
    out = R.forward(p, x, train=False)
    _close(out["mu"], golden["g1_mu"], 1e-5, 1e-6, "mu")
    _close(out["logvar"], golden["g1_logvar"], 1e-5, 1e-6, "logvar")
    _close(out["u"], golden["g1_u"], 1e-5, 1e-5, "u")
    _close(out["scores"], golden["g1_scores"], 1e-5, 3e-5, "scores")
    loss = R.vae_loss(out["scores"], x, out["mu"], out["logvar"], c["beta"])
    _close([t.item() for t in loss], golden["g1_loss"], 1e-5, 1e-6, "loss")
    top = np.stack([np.argsort(r, kind="stable")[::-1][:10] for r in out["scores"].numpy()])
    # bit-exact unless the reference scores themselves tie within fp32 noise
    assert (top == golden["g1_top10"]).mean() > 0.99


@pytest.mark.parametrize("name", sorted(TRAIN_CONFIGS))
def test_train_steps(golden, name):
    c = TRAIN_CONFIGS[name]
    X = synth_csr(c["n_users"], c["n_items"], lam=c.get("lam", 3.0), seed=200 + c["seed"])
    E = synth_embeddings(c["n_items"], c["d"], seed=300 + c["seed"])
    p = R.init_params(c["n_items"], E, c["latent"], c["hidden"], seed=c["seed"])
    x = torch.as_tensor(X.toarray(), dtype=torch.float32)
    state = {}
    has_proj = c["latent"] != c["d"]
    for step in (1, 2):
        g = lambda k: torch.as_tensor(golden[f"g2{name}_s{step}_{k}"])
        enc = [g(f"encmask{k}") for k in range(len(c["hidden"]))]
        proj = g("projmask") if has_proj else None
        r = R.train_step(p, state, x, c["beta"], lr=c["lr"], weight_decay=c.get("wd", 0.0), enc_masks=enc,
                         proj_mask=proj, eps=g("eps"))
        _close(r["loss"], golden[f"g2{name}_loss"][step - 1], 1e-5, 1e-6, f"loss step {step}")
        _close(r["total_norm"], golden[f"g2{name}_norm"][step - 1], 1e-5, 1e-7, f"norm step {step}")
        if step == 1:
            for n, gr in r["grads"].items():
                _close_max(gr, golden[f"g2{name}_s1_grad_{n}"], 1e-5, f"grad {n}")
    for n in R.param_names(p):
        # Adam turns near-zero gradients into O(lr) steps, so params get a looser bound
        _close_max(p[n], golden[f"g2{name}_s2_param_{n}"], 2e-4, f"param {n}")
        _close_max(state[n][0], golden[f"g2{name}_s2_m_{n}"], 1e-5, f"m {n}")
        _close_max(state[n][1], golden[f"g2{name}_s2_v_{n}"], 1e-5, f"v {n}")


@pytest.mark.parametrize("name", sorted(TRAIN_CONFIGS))
def test_cpu_trainer_steps(golden, name):
    """The module-based CPU trainer (bench.py's cpu_baseline) takes the reference's steps too."""
    c = TRAIN_CONFIGS[name]
    X = synth_csr(c["n_users"], c["n_items"], lam=c.get("lam", 3.0), seed=200 + c["seed"])
    E = synth_embeddings(c["n_items"], c["d"], seed=300 + c["seed"])
    p = R.init_params(c["n_items"], E, c["latent"], c["hidden"], seed=c["seed"])
    x = torch.as_tensor(X.toarray(), dtype=torch.float32)
    tr = R.CpuTrainer(p, c.get("dropout", 0.3), lr=c["lr"], weight_decay=c.get("wd", 0.0))
    has_proj = c["latent"] != c["d"]
    for step in (1, 2):
        g = lambda k: torch.as_tensor(golden[f"g2{name}_s{step}_{k}"])
        enc = [g(f"encmask{k}") for k in range(len(c["hidden"]))]
        loss = tr.step(x, c["beta"], enc_masks=enc, proj_mask=g("projmask") if has_proj else None, eps=g("eps"))
        _close(loss, golden[f"g2{name}_loss"][step - 1][0], 1e-5, 1e-6, f"loss step {step}")
    st = tr.state()
    for n in R.param_names(p):
        _close_max(st[n], golden[f"g2{name}_s2_param_{n}"], 2e-4, f"param {n}")


def test_metric_kats(golden):
    for trial, k, rec, ndcg, hr in golden["g3_kat"]:
        recd, rel = golden[f"g3_rec_{int(trial)}"], golden[f"g3_rel_{int(trial)}"]
        k = int(k)
        assert R.recall_at_k(recd, rel, k) == pytest.approx(rec, abs=1e-12)
        assert R.ndcg_at_k(recd, rel, k) == pytest.approx(ndcg, abs=1e-12)
        assert R.hit_ratio_at_k(recd, rel, k) == pytest.approx(hr, abs=1e-12)


def test_eval_protocol(golden):
    c = EVAL_CONFIG
    X = synth_csr(c["n_users"], c["n_items"], seed=100)
    s = golden["g1_scores"]
    res = {k: [] for k in (5, 10, 20)}
    for i, (t, negs) in enumerate(zip(golden["g4_test_items"], golden["g4_negatives"])):
        cand = np.concatenate([[t], negs])
        ranked = R.rank_candidates(s[i], cand)
        for k in res:
            res[k].append([R.recall_at_k(ranked, [t], k), R.ndcg_at_k(ranked, [t], k), R.hit_ratio_at_k(ranked, [t], k)])
    got = np.array([np.mean(res[k], axis=0) for k in (5, 10, 20)])
    np.testing.assert_allclose(got, golden["g4_metrics"], atol=1e-12)
    for i in range(8):
        top = R.topk_exclude_seen(s[i], X[i].indices, 20)
        np.testing.assert_array_equal(top, golden["g4_full_top20"][i])


def test_csr_semantics(golden):
    df = pd.DataFrame({
        "user_id": ["a", "a", "b", "b", "b", "c", "c", "a", "d"],
        "asin": ["x", "x", "y", "z", "y", "x", "w", "w", "z"],
        "binary_rating": [1, 1, 1, 0, 1, 0, 1, 1, 0],
    })
    u2i = {u: i for i, u in enumerate("abcd")}
    i2i = {a: i for i, a in enumerate("wxyz")}
    M = R.build_matrix(df.user_id.map(u2i).values, df.asin.map(i2i).values, df.binary_rating.values, (4, 4))
    np.testing.assert_array_equal(M.toarray(), golden["g5_train_dense"])
    assert golden["g5_train_dense"].max() == 2.0  # duplicates are summed, not binarised
