"""In-process A/B of whole train steps: one dataset, several arms (environment settings the executor reads when a
FusedTrainer is built or a step graph is captured), interleaved over rounds, each arm on a fresh trainer.

    python scripts/bench_step_ab.py --workload syn1m --arm base: --arm k8:HVAE_STEPS_PER_GRAPH=8 [--rounds 2]

Prints one JSON line per (round, arm): ms per step over --steps graph-replayed steps after --warmup, the same
timing as bench.py's (synchronise, wall clock, synchronise).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "recommendation-system_amd"), str(ROOT / "tests" / "golden")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syn1m", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--arm", action="append", required=True, help="NAME:ENV=VAL,ENV=VAL (empty settings allowed)")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    args = ap.parse_args()
    from hvae.executor import ConstBeta, FusedTrainer
    from src.ml.model import HybridVAE
    w = dict(bench.WORKLOADS[args.workload])
    X, E, users = bench.make_data(w, 0, 1)
    dev = torch.device("cuda", 0)
    B = w["batch"]
    n_per_epoch = len(users) // B
    arms = []
    for a in args.arm:
        name, _, kv = a.partition(":")
        env = dict(p.split("=", 1) for p in kv.split(",") if p)
        arms.append((name, env))
    for rnd in range(args.rounds):
        for name, env in arms:
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                torch.manual_seed(0)
                model = HybridVAE(w["items"], E, latent_dim=w["latent"], hidden_dims=w["hidden"],
                                  dropout=w["dropout"], beta=w["beta"]).to(dev)
                fused = FusedTrainer(model, dev, lr=w["lr"], precision=args.precision, seed=1234, use_graphs=True)
                data = fused.device_data(X, users)
                gen = torch.Generator(device=dev).manual_seed(0)
                beta = ConstBeta(w["beta"])

                def run(nsteps):
                    done = 0
                    while done < nsteps:
                        k = min(nsteps - done, n_per_epoch)
                        fused.run_epoch(data, B, True, beta, w["dropout"], generator=gen, max_batches=k)
                        done += k

                run(args.warmup)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(args.steps)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / args.steps * 1e3
                print(json.dumps({"workload": args.workload, "precision": args.precision, "round": rnd,
                                  "arm": name, "env": env, "ms_per_step": round(ms, 4),
                                  "users_per_s": round(B / ms * 1e3, 1)}), flush=True)
                del fused, model, data
                torch.cuda.empty_cache()
            finally:
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v


if __name__ == "__main__":
    main()
