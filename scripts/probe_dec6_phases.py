"""Phase anatomy of the version-6 bf16 sweep from a timing build (DEC6_TIMING=1, outputs unchanged, one s_memtime
per phase boundary): per wave, the cycles of the sweep loop spent waiting at [L] (tile landed, P published), in
phase 1 (GEMM1 | GEMM2 first half | DMA), at put + [B1], and in phase 2 (GEMM2 second half | softmax), per tile.

    HVAE_LIB=build_var/libhvae_d6tm.so python scripts/probe_dec6_phases.py [--nb 4096] [--N 1000000]
"""
import os
os.environ.setdefault("HVAE_DEC_V6", "1")  # version 6 is an A/B-library sweep (HVAE_LIB=build_var/libhvae_ab.so or a variant)
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hvae import ops  # noqa: E402
from hvae._lib import check, lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nb", type=int, default=4096)
ap.add_argument("--N", type=int, default=1000000)
args = ap.parse_args()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
E = torch.randn(args.N, 768, device=dev, generator=g)
E /= E.norm(dim=1, keepdim=True)
U = torch.randn(args.nb, 768, device=dev, generator=g) * (4.0 / 768 ** 0.5)
img = ops.decoder_image(E)
en = ops.row_norm_max(img)
del E
L = lib()
fetch = L.hvae_dec6_timing_fetch
fetch.argtypes = [C.c_void_p]
fetch.restype = C.c_int
for rep in range(3):
    lse, O = ops.decoder_fwd(U, img, en)
    torch.cuda.synchronize()
    buf = np.zeros((1024, 8), dtype=np.uint64)
    check(fetch(buf.ctypes.data), "hvae_dec6_timing_fetch")
    tiles = buf[:, 4].astype(np.float64)
    live = tiles > 0
    t = buf[live, :6].astype(np.float64)
    per = t[:, :4].sum(0) / t[:, 4].sum()
    loop = t[:, :4].sum(1)
    out = {"rep": rep, "waves": int(live.sum()), "tiles_per_wave_mean": float(tiles[live].mean()),
           "cycles_per_tile": {k: round(float(v), 1) for k, v in zip(["wait_L", "phase1", "put_B1", "phase2"], per)},
           "loop_cycles_per_tile": round(float(per.sum()), 1),
           "kernel_cycles_max": float(t[:, 5].max()), "kernel_cycles_mean": float(t[:, 5].mean()),
           "loop_cycles_max": float(loop.max()), "loop_cycles_min": float(loop.min())}
    print(json.dumps(out), flush=True)
