"""Debug: run the version-6 sweep through hvae_decoder_fwd with a workspace poisoned with 0xFF bytes, for each
shape NBxN given, and report the partial slot rows that come back unwritten or flagged (a flagged user is
recomputed exactly by the finalize, so a sweep that flags users gives right answers slowly), and lse against
float64 for the unflagged users."""
import os
os.environ.setdefault("HVAE_DEC_V6", "1")  # version 6 is an A/B-library sweep (HVAE_LIB=build_var/libhvae_ab.so or a variant)
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd")]
import torch
from hvae import ops
from hvae._lib import lib, ptr, check, stream_of
dev = torch.device("cuda", 0)
D = 768


def plan(nb, N):
    ntiles = -(-N // 32); nub = -(-nb // 96)
    S = -(-256 // nub); S = max(1, min(S, max(1, ntiles // 8))); tps = -(-ntiles // S); S = -(-ntiles // tps)
    tot = nub * S
    main, X = (tot, 0) if tot <= 256 else (256, tot - 256)
    P = 256 // X if X else 0
    return dict(nub=nub, S=S, tps=tps, main=main, X=X, P=P, slots=main + X * P)


def run(nb, N, calls=2):
    g = torch.Generator(device=dev).manual_seed(0)
    E = torch.randn(N, D, device=dev, generator=g)
    E /= E.norm(dim=1, keepdim=True)
    U = torch.randn(nb, D, device=dev, generator=g) * (4.0 / D ** 0.5)
    img = ops.decoder_image(E)
    en = ops.row_norm_max(img)
    dt, _, Eh = ops._dec_operand(img)
    need = lib().hvae_decoder_workspace(dt, nb, N, D)
    pl = plan(nb, N)
    rows = pl["slots"] * 96
    S64 = U.bfloat16().double() @ img.bf16.double().t()
    lref = torch.logsumexp(S64, 1)
    for call in range(calls):
        ws = torch.full((need,), 0xFF, dtype=torch.uint8, device=dev)
        lse = torch.empty(nb, device=dev); O = torch.empty(nb, D, device=dev)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        check(lib().hvae_decoder_fwd(dt, ptr(U), U.stride(0), ptr(Eh), ptr(en), nb, N, D, ptr(lse), ptr(O), ptr(ws),
                                     ws.numel(), stream_of(U)), "fwd")
        torch.cuda.synchronize(); ms = (time.perf_counter() - t0) * 1e3
        fb = -(-rows * 4 // 256) * 256
        flag = ws[:rows * 4].view(torch.int32)
        m = ws[fb:fb + rows * 4].view(torch.float32)
        l = ws[fb + rows * 4:fb + rows * 8].view(torch.float32)
        bad = torch.nonzero(flag != 0).flatten().tolist()
        print(f"nb {nb} N {N} plan {pl} call {call}: {ms:.2f} ms; rows with flag != 0: {len(bad)}; "
              f"lse max err {float((lse.double() - lref).abs().max()):.3e}", flush=True)
        for r in bad[:6]:
            print("   row", r, "slot", r // 96, "j", r % 96, "flag", int(flag[r]), "m", float(m[r]), "l", float(l[r]),
                  flush=True)


for a in sys.argv[1:]:
    nb, N = (int(v) for v in a.split("x"))
    run(nb, N)
