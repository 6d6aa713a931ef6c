"""Paired calibration of bench.py's CPU baseline against the reference trainer (build container only).

    PYTHONDONTWRITEBYTECODE=1 python scripts/calibrate_cpu_baseline.py [--threads 8] [--rounds 6]

Imports the reference's own src/ml (the two absent third-party imports stubbed, as
tests/golden/make_golden.py does) and times, interleaved round by round in one process, one
VAETrainer.train_epoch step of the reference and one oracle.ref_cpu.CpuTrainer.step on the same
All_Beauty-shaped batches (B = 64, 8 threads). Interleaving cancels the host's load swings, which make
unpaired timings here vary 3x; the ratio of medians (and of the best rounds) is the calibration. Writes one JSON line.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden")]

import torch  # noqa: E402

from gen import synth_csr, synth_embeddings  # noqa: E402
from make_golden import import_reference  # noqa: E402
from oracle import ref_cpu as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=15)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    model_m, train_m, _ = import_reference()
    U, N, d, L, H, B = 22363, 12101, 384, 128, [512], 64
    X = synth_csr(U, N, lam=3.0, seed=0)
    E = synth_embeddings(N, d, seed=1)
    torch.manual_seed(0)
    ref_model = model_m.HybridVAE(N, E, latent_dim=L, hidden_dims=H, dropout=0.3, beta=0.2)
    ref_tr = train_m.VAETrainer(ref_model, torch.device("cpu"), lr=1e-3)
    ours = R.CpuTrainer(R.init_params(N, E, L, H, seed=0), 0.3, lr=1e-3)
    batches = [torch.as_tensor(X[i * B:(i + 1) * B].toarray(), dtype=torch.float32) for i in range(args.steps)]

    class Once:  # a one-batch loader for VAETrainer.train_epoch
        def __init__(self, x):
            self.x = x

        def __iter__(self):
            return iter([self.x])

        def __len__(self):
            return 1

    import tqdm
    tqdm.tqdm = lambda it, **k: it  # the reference wraps its loader in tqdm; keep the timing free of it
    train_m.tqdm = tqdm.tqdm
    t_ref, t_ours = [], []
    for x in batches[:2]:  # warm-up
        ref_tr.train_epoch(Once(x))
        ours.step(x, 0.2)
    for _ in range(args.rounds):
        t0 = time.perf_counter()
        for x in batches:
            ref_tr.train_epoch(Once(x))
        t1 = time.perf_counter()
        for x in batches:
            ours.step(x, 0.2)
        t2 = time.perf_counter()
        t_ref.append((t1 - t0) / len(batches))
        t_ours.append((t2 - t1) / len(batches))
    mr, mo = statistics.median(t_ref), statistics.median(t_ours)
    print(json.dumps({"shape": "All_Beauty 22,363 x 12,101, d 384, L 128, H [512], B 64", "threads": args.threads,
                      "reference_step_ms_median": round(mr * 1e3, 2), "cpu_trainer_step_ms_median": round(mo * 1e3, 2),
                      "ratio_cpu_trainer_over_reference": round(mo / mr, 3),
                      "ratio_of_best_rounds": round(min(t_ours) / min(t_ref), 3),
                      "reference_users_per_s": round(B / mr, 1), "cpu_trainer_users_per_s": round(B / mo, 1),
                      "rounds_ms": {"reference": [round(t * 1e3, 2) for t in t_ref],
                                    "cpu_trainer": [round(t * 1e3, 2) for t in t_ours]}}))


if __name__ == "__main__":
    main()
