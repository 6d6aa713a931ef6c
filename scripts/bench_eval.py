"""Eval / serving throughput on MI355X (users/s), beside the reference's measured 374 users/s (CPU,
All_Beauty, 99-negative protocol of src/ml/evaluate.py:149-215).

    python scripts/bench_eval.py [--workload all_beauty|syn1m|syn10m] [--batch 1024] [--k 20] [--reps 5]

Lines (JSON, one per measurement):
  * topk_fused     full-ranking top-k of a batch of users (seen items excluded): encoder -> u -> hvae_topk_fused
                   (bf16 MFMA shortlist + fp32 rescore, no [B, N] scores); the /recommend/batch core;
  * topk_matrix    the same answer through the fp32 [B, N] score matrix (hvae_gemm_f32) + hvae_topk;
  * neg99          RecommendationEvaluator.evaluate_dataset_with_negatives (1 test item + 99 sampled negatives per
                   user; host-side numpy sampling included, as in the reference).
Random-init weights of the workload's shape, synthetic interactions (tests/golden/gen.py).
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd"), str(ROOT / "tests" / "golden")]

import torch  # noqa: E402

WORKLOADS = {
    "all_beauty": dict(users=22363, items=12101, d=384, lam=3.0),
    "syn1m": dict(users=200000, items=100000, d=384, lam=15.0),
    "syn10m": dict(users=200000, items=1000000, d=768, lam=15.0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="all_beauty", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--neg99-users", type=int, default=4096)
    ap.add_argument("--skip-matrix", action="store_true")
    ap.add_argument("--probes", nargs="*", default=None, help="only these score arms (topk_fused, ...)")
    args = ap.parse_args()
    from gen import synth_csr
    from hvae import ops
    from src.ml.evaluate import RecommendationEvaluator
    from src.ml.model import HybridVAE

    w = WORKLOADS[args.workload]
    dev = torch.device("cuda", 0)
    X = synth_csr(w["users"], w["items"], lam=w["lam"], seed=1)
    g = torch.Generator(device=dev).manual_seed(0)
    E = torch.randn(w["items"], w["d"], device=dev, generator=g)
    E /= E.norm(dim=1, keepdim=True)
    torch.manual_seed(0)
    model = HybridVAE(w["items"], E.cpu().numpy(), latent_dim=128, hidden_dims=[512], dropout=0.3,
                      beta=0.2).to(dev).eval()
    csr = ops.csr_from_scipy(X, dev)
    rng = np.random.default_rng(0)
    B, k = args.batch, args.k

    def batch_rows():
        return torch.as_tensor(rng.choice(w["users"], B, replace=False).astype(np.int32), device=dev)

    def run_fused(rows):
        c = ops.Csr(csr.row_ptr, csr.col_idx, csr.vals, w["items"], rows=rows)
        u = model.user_vectors(c)
        return model.topk_scores(u, k, exclude=c)

    def run_matrix(rows):
        c = ops.Csr(csr.row_ptr, csr.col_idx, csr.vals, w["items"], rows=rows)
        u = model.user_vectors(c)
        S = ops.gemm(u, model.item_embeddings.t())
        return ops.topk(S, k, exclude=c)

    import os

    def run_fused_global(rows):  # A/B: the scan reading E fragments straight from global memory
        os.environ["HVAE_TOPK_LDS"] = "0"
        try:
            return run_fused(rows)
        finally:
            os.environ.pop("HVAE_TOPK_LDS")

    arms = [("topk_fused", run_fused), ("topk_fused_global_scan", run_fused_global)] + \
        ([] if args.skip_matrix else [("topk_matrix", run_matrix)])
    if args.probes:
        arms = [a for a in arms if a[0] in args.probes]
    res = {}
    rows = [batch_rows() for _ in range(args.reps)]  # the same batches for every arm
    for name, fn in arms:
        fn(batch_rows())  # warm-up: kernel load, caches
        torch.cuda.synchronize()
        t = time.perf_counter()
        outs = [fn(r) for r in rows]
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / args.reps
        res[name] = outs
        print(json.dumps({"workload": args.workload, "probe": name, "batch": B, "k": k, "items": w["items"],
                          "d": w["d"], "ms_per_batch": round(dt * 1e3, 3), "users_per_s": round(B / dt, 1)}),
              flush=True)
    if "topk_matrix" in res:
        same = np.mean([(a[0].cpu() == b[0].cpu()).float().mean().item()
                        for a, b in zip(res["topk_fused"], res["topk_matrix"])])
        print(json.dumps({"workload": args.workload, "probe": "fused_vs_matrix_index_agreement",
                          "fraction": round(float(same), 6)}), flush=True)

    # 99-negative protocol (reference's headline eval)
    if args.neg99_users:
        import pandas as pd
        n = min(args.neg99_users, w["users"])
        users = rng.choice(w["users"], n, replace=False)
        u2i = {f"u{i}": i for i in range(w["users"])}
        i2i = {f"i{j}": j for j in range(w["items"])}
        tests = [f"i{int(rng.integers(w['items']))}" for _ in users]
        test_df = pd.DataFrame({"user_id": [f"u{i}" for i in users], "asin": tests})
        ev = RecommendationEvaluator(model, X, u2i, i2i, dev, batch_size=1024)
        np.random.seed(0)
        ev.evaluate_dataset_with_negatives(test_df.head(256), n_negatives=99)  # warm-up
        torch.cuda.synchronize()
        np.random.seed(0)
        t = time.perf_counter()
        ev.evaluate_dataset_with_negatives(test_df, n_negatives=99)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(json.dumps({"workload": args.workload, "probe": "neg99", "users": n, "s": round(dt, 3),
                          "users_per_s": round(n / dt, 1), "reference_cpu_users_per_s": 374}), flush=True)


if __name__ == "__main__":
    main()
