"""Per-tile cycle budget of the product bf16 sweep (k_dec5_bf16, version 5) from a timing build (DEC5_TIMING=1: one
s_memtime per phase boundary, outputs unchanged).

Per wave role, the cycles per tile of the sweep loop spent
  producer: waiting for its own LDS-DMA pieces (vmcnt) | at the tile barrier | GEMM1 with its pieces | tail mask,
            exponentials and P out;
  consumer: waiting for its pieces | at the barrier | P read and GEMM2 with its pieces;
plus the kernel's cycles, the in-kernel clock (s_memtime / s_memrealtime x 100 MHz) and the sweep's wall time
(hipEvents around each launch, the build's probe bracket).

    HVAE_LIB=build_var/libhvae_d5tm.so python scripts/probe_dec5_phases.py [--nb 4096] [--N 1000000] [--label x]
"""
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
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--label", default="")
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
fetch = getattr(L, "hvae_dec5_timing_fetch", None)
if fetch is not None:
    fetch.argtypes = [C.c_void_p]
    fetch.restype = C.c_int
ops.decoder_fwd(U, img, en)  # warm-up: kernel attributes, clocks
torch.cuda.synchronize()
for rep in range(args.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    lse, O = ops.decoder_fwd(U, img, en)
    e1.record()
    torch.cuda.synchronize()
    out = {"label": args.label, "rep": rep, "nb": args.nb, "N": args.N, "wall_ms": round(e0.elapsed_time(e1), 3),
           "flagged_or_nan": int((~torch.isfinite(lse)).sum().item())}
    if fetch is not None:
        buf = np.zeros((2048, 8), dtype=np.uint64)
        check(fetch(buf.ctypes.data), "hvae_dec5_timing_fetch")
        live = buf[:, 4] > 0
        for role, name, cols in ((0, "producer", ["wait_vm", "barrier", "gemm1_dma", "softmax_p_out"]),
                                 (1, "consumer", ["wait_vm", "barrier", "gemm2_dma"])):
            sel = live & (buf[:, 7] == role)
            t = buf[sel].astype(np.float64)
            per = t[:, :4].sum(0) / t[:, 4].sum()
            out[name] = {k: round(float(v), 1) for k, v in zip(cols, per)}
            out[name]["loop_per_tile"] = round(float(per[:len(cols)].sum()), 1)
            out[name]["waves"] = int(sel.sum())
        t = buf[live].astype(np.float64)
        ghz = t[:, 5] / (t[:, 6] / 100e6) / 1e9
        out["kernel_cycles_mean"] = float(t[:, 5].mean())
        out["tiles_per_wave_mean"] = float(t[:, 4].mean())
        out["clock_ghz_median"] = round(float(np.median(ghz)), 3)
        out["kernel_cycles_per_tile"] = round(float(t[:, 5].mean() / t[:, 4].mean()), 1)
    print(json.dumps(out), flush=True)
