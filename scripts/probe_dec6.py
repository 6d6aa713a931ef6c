"""Time the d = 768 bf16 sweep (A/B library or a variant build, HVAE_DEC_V6=1: version 6 above 64 users) over growing item counts, one line
per call, so that a slow or stuck shape shows where it starts."""
import os
os.environ.setdefault("HVAE_DEC_V6", "1")  # version 6 is an A/B-library sweep (HVAE_LIB=build_var/libhvae_ab.so or a variant)
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd")]
import torch
from hvae import ops
dev = torch.device("cuda", 0)
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
for N in [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["200000", "400000", "1000000"])]:
    g = torch.Generator(device=dev).manual_seed(0)
    E = torch.randn(N, 768, device=dev, generator=g)
    E /= E.norm(dim=1, keepdim=True)
    U = torch.randn(nb, 768, device=dev, generator=g) * (4.0 / 768 ** 0.5)
    img = ops.decoder_image(E)
    en = ops.row_norm_max(img)
    del E
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lse, O = ops.decoder_fwd(U, img, en)
        torch.cuda.synchronize()
        print(f"nb {nb} N {N} rep {rep}: {(time.perf_counter() - t0) * 1e3:.2f} ms finite {bool(torch.isfinite(lse).all())}",
              flush=True)
    del img, lse, O
