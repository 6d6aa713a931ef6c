"""Per-launch timing of the row-parallel latent / projection MLP (hvae_mlp_fwd_rows / hvae_mlp_bwd_rows /
hvae_gemm_f32_multi) at the train-step shapes, with the library's hipEvent probe.

    python scripts/bench_mlp_rows.py [--reps 200] [--batches 64,512,1024] [--d 384]
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd"), str(ROOT / "tests"), str(ROOT / "tests" / "golden"), str(ROOT)]

import torch  # noqa: E402

from hvae._lib import check, lib  # noqa: E402
from test_gpu_mlp_rows import _args, _setup  # noqa: E402


def probe(name, fn, reps):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    check(lib().hvae_probe_arm(name.encode(), reps), "arm")
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    avg, n = C.c_double(), C.c_int()
    check(lib().hvae_probe_collect(C.byref(avg), C.byref(n)), "collect")
    check(lib().hvae_probe_arm(None, 0), "disarm")
    return round(avg.value, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--batches", default="64,512,1024")
    ap.add_argument("--d", type=int, default=384)
    ap.add_argument("--shapes", default=None,
                    help="H:L:D list (e.g. 512:128:384,32:32:384) timed at the first batch instead of --d")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.shapes:
        B = int(args.batches.split(",")[0])
        for sh in args.shapes.split(","):
            H, L, D = (int(v) for v in sh.split(":"))
            t, d, out = _setup(B, H, L, D, dev, 1)
            a = _args(B, H, L, D, d, out, True, 0.3, explicit=False, seed=3)
            fwd = probe("mlp_fwd", lambda: check(lib().hvae_mlp_fwd_rows(C.byref(a), None), "fwd"), args.reps)
            bwd = probe("mlp_bwd", lambda: check(lib().hvae_mlp_bwd_rows(C.byref(a), None), "bwd"), args.reps)
            print(json.dumps({"B": B, "H": H, "L": L, "D": D, "fwd_us": fwd, "bwd_us": bwd,
                              "weight_bytes": 4 * (2 * L * H + D * L + D * D)}), flush=True)
        return
    H, L, D = 512, 128, args.d
    for B in (int(b) for b in args.batches.split(",")):
        t, d, out = _setup(B, H, L, D, dev, 1)
        a = _args(B, H, L, D, d, out, True, 0.3, explicit=False, seed=3)
        fwd = probe("mlp_fwd", lambda: check(lib().hvae_mlp_fwd_rows(C.byref(a), None), "fwd"), args.reps)
        bwd = probe("mlp_bwd", lambda: check(lib().hvae_mlp_bwd_rows(C.byref(a), None), "bwd"), args.reps)
        wbytes = 4 * (2 * L * H + D * L + D * D)
        print(json.dumps({"B": B, "H": H, "L": L, "D": D, "fwd_us": fwd, "bwd_us": bwd,
                          "weight_bytes": wbytes}), flush=True)


if __name__ == "__main__":
    main()
