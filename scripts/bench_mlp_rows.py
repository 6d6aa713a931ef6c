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
    ap.add_argument("--fused", action="store_true", help="time the step's composition (encoder layer, plan block, "
                    "LayerNorm backward) at the first batch")
    ap.add_argument("--lam", type=float, default=3.0, help="--fused: synth_csr lam (All_Beauty: 3)")
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
    if args.fused:
        # the step's composition at the first batch: + the fused encoder layer (enc_x), + the plan block (plan_x),
        # + the backward's LayerNorm (ln_w), on an All_Beauty-like CSR batch
        from gen import synth_csr
        from hvae import _lib, ops
        from hvae._lib import ptr
        B = int(args.batches.split(",")[0])
        N = 12101
        X = synth_csr(B, N, lam=args.lam, seed=5)
        xd = ops.csr_from_scipy(X, dev)
        g = torch.Generator().manual_seed(9)
        w1t = (torch.randn(N, H, generator=g) * 0.05).to(dev)
        b1, lnw, lnb = (torch.randn(H, generator=g) * 0.1).to(dev), (1 + 0.1 * torch.randn(H, generator=g)).to(dev), \
            (0.1 * torch.randn(H, generator=g)).to(dev)
        h, xhat, rstd = torch.empty(B, H, device=dev), torch.empty(B, H, device=dev), torch.empty(B, device=dev)
        rg = ops.RowGradBuffers(N, H, max(int(X.nnz), 1), dev)
        da, dw, db, dbias = (torch.empty(B, H, device=dev), torch.empty(H, device=dev), torch.empty(H, device=dev),
                             torch.empty(H, device=dev))
        ws = torch.empty(max(int(lib().hvae_mlp_bwd_rows_workspace(B, H)), 256), dtype=torch.uint8, device=dev)
        for enc in (0, 1):
            for plan in (0, 1):
                t, d, out = _setup(B, H, L, D, dev, 1)
                a = _args(B, H, L, D, d, out, True, 0.3, explicit=False, seed=3)
                if enc:
                    a.enc_x, a.w1t, a.b1, a.ln_w, a.ln_b = C.pointer(xd.struct), ptr(w1t), ptr(b1), ptr(lnw), ptr(lnb)
                    a.h, a.xhat, a.rstd = ptr(h), ptr(xhat), ptr(rstd)
                if plan:
                    a.plan_x, a.plan_rg = C.pointer(xd.struct), C.pointer(rg.struct)
                fwd = probe("mlp_fwd", lambda: check(lib().hvae_mlp_fwd_rows(C.byref(a), None), "fwd"), args.reps)
                print(json.dumps({"B": B, "nnz": int(X.nnz), "enc": enc, "plan": plan, "fwd_us": fwd}), flush=True)
        for ln in (0, 1):
            t, d, out = _setup(B, H, L, D, dev, 1)
            a = _args(B, H, L, D, d, out, True, 0.3, explicit=False, seed=3)
            check(lib().hvae_mlp_fwd_rows(C.byref(a), None), "fwd")
            if ln:
                xhat.normal_()
                rstd.uniform_(0.5, 1.5)
                a.ln_w, a.ln_b, a.xhat, a.rstd, a.enc_layer = ptr(lnw), ptr(lnb), ptr(xhat), ptr(rstd), 0
                a.da, a.d_ln_w, a.d_ln_b, a.d_bias, a.ws, a.ws_bytes = ptr(da), ptr(dw), ptr(db), ptr(dbias), ptr(ws), ws.numel()
            bwd = probe("mlp_bwd", lambda: check(lib().hvae_mlp_bwd_rows(C.byref(a), None), "bwd"), args.reps)
            print(json.dumps({"B": B, "ln": ln, "bwd_us": bwd}), flush=True)
        return
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
