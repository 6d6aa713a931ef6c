"""Debug helper: lazy vs dense Adam, step by step, on the shape of test_lazy_adam_is_bitwise_dense.

Prints the first step at which the flat parameters differ and which segment (W1t rows or the dense
small parameters) does, plus the step-table constants against a host (numpy float64) evaluation.
"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd"), str(ROOT / "tests" / "golden")]

from gen import synth_csr, synth_embeddings  # noqa: E402
from hvae.executor import ConstBeta, FusedTrainer  # noqa: E402
from src.ml.model import HybridVAE  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    X = synth_csr(290, 700, seed=13)
    E = synth_embeddings(700, 128, seed=14)
    runs = {}
    for lazy in (False, True):
        torch.manual_seed(0)
        model = HybridVAE(700, E, latent_dim=64, hidden_dims=[128], dropout=0.3, beta=0.2).to(dev)
        fused = FusedTrainer(model, dev, weight_decay=0.0, precision="bf16", seed=77, use_graphs=False)
        fused.lazy_adam = lazy
        data = fused.device_data(X, list(range(290)))
        snaps = []
        for k in range(4):
            fused.run_epoch(data, 32, True, ConstBeta(0.2), 0.3, generator=torch.Generator().manual_seed(6 + k),
                            max_batches=1)
            snaps.append((fused.flat.clone(), fused.m.clone(), fused.v.clone()))
        runs[lazy] = (snaps, fused)
    lay = runs[True][1].layout
    n_w1 = lay.small_offset
    for k in range(4):
        a, b = runs[False][0][k], runs[True][0][k]
        for name, x, y in zip("pmv", a, b):
            dw = (x[:n_w1] != y[:n_w1]).sum().item()
            ds = (x[n_w1:] != y[n_w1:]).sum().item()
            print(f"step {k + 1} {name}: W1t differ {dw}, dense differ {ds}", flush=True)
    tab = runs[True][1].adam_tab.view(-1, 2)[:6].cpu().numpy()
    lr, (b1, b2) = runs[True][1].lr, runs[True][1].betas
    for t in range(1, 5):
        host = (np.float32(lr / (1.0 - b1 ** t)), np.float32(np.sqrt(1.0 - b2 ** t)))
        print(f"tab[{t}] = {tab[t].tolist()} host {host}", flush=True)


if __name__ == "__main__":
    main()
