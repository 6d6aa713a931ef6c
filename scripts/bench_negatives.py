"""The 99-negative sampler alone (hvae_negatives_legacy, host code): rows/s of ops.negatives_legacy for the
evaluation workloads' shapes, in the AVX-512 and the scalar form of the draw loop and at several worker counts.
Synthetic interactions (tests/golden/gen.py); one JSON line per arm.
Reference: src/ml/evaluate.py:149-185 (one np.random.choice per row)."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd"), str(ROOT / "tests" / "golden")]

WORKLOADS = {"all_beauty": (22363, 12101, 3.0, 4096), "syn1m": (200000, 100000, 15.0, 1024)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", nargs="*", default=sorted(WORKLOADS))
    ap.add_argument("--workers", nargs="*", type=int, default=[1, 4, 8, 12])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from gen import synth_csr
    from hvae import ops
    for wl in args.workloads:
        U, I, lam, n = WORKLOADS[wl]
        X = synth_csr(U, I, lam=lam, seed=1).tocsr()
        rng = np.random.default_rng(0)
        users = rng.choice(U, n, replace=False)
        tests = rng.integers(I, size=n)
        ref = None
        for form in ("simd", "scalar"):
            os.environ["HVAE_NEG_SCALAR"] = "1" if form == "scalar" else "0"
            for w in args.workers:
                os.environ["HVAE_NEG_WORKERS"] = str(w)
                np.random.seed(0)
                ops.negatives_legacy(X.indptr, X.indices, I, users[:64], tests[:64], 99)  # warm-up
                best = 1e9
                for _ in range(args.reps):
                    np.random.seed(0)
                    t = time.perf_counter()
                    got = ops.negatives_legacy(X.indptr, X.indices, I, users, tests, 99)
                    best = min(best, time.perf_counter() - t)
                if ref is None:
                    ref = got
                same = all(np.array_equal(a, b) for a, b in zip(got, ref))
                print(json.dumps({"workload": wl, "items": I, "rows": n, "form": form, "workers": w,
                                  "s": round(best, 4), "rows_per_s": round(n / best, 1), "same_as_first": same}),
                      flush=True)


if __name__ == "__main__":
    main()
