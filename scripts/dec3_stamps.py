"""Read the per-wave phase sums of a DEC3_STAMPS=1 build (scripts/build_variant.sh stamps -DDEC3_STAMPS=1)
after one d = 768 sweep, and print the mean s_memtime ticks per tile of each loop phase.

    HVAE_LIB=build_var/libhvae_stamps.so python scripts/dec3_stamps.py [--nb 4096 --N 1000000]
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd")]
import torch  # noqa: E402

from hvae import ops  # noqa: E402
from hvae._lib import check, lib  # noqa: E402

PHASES = ["loop_tail", "dma_wait", "barrier_A", "gemm1_softmax_dma", "p_out_barrier_B", "halfS_out_gemm2_own",
          "gemm2_partner"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb", type=int, default=4096)
    ap.add_argument("--N", type=int, default=1_000_000)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    E32 = torch.randn(args.N, 768, device=dev, generator=g)
    E32 /= E32.norm(dim=1, keepdim=True)
    U = torch.randn(args.nb, 768, device=dev, generator=g) * (4.0 / 768 ** 0.5)
    E = ops.decoder_image(E32)
    enorm = ops.row_norm_max(E)
    for _ in range(3):
        ops.decoder_fwd(U, E, enorm)
    torch.cuda.synchronize()
    buf = np.zeros((4096, 8), dtype=np.uint64)
    f = lib().hvae_debug_dec3_stamps
    f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_size_t]
    check(f(buf.ctypes.data, buf.nbytes), "stamps")
    live = buf[buf[:, 7] > 0]
    tiles = live[:, 7].astype(np.float64)
    per = {p: float(np.mean(live[:, i] / tiles)) for i, p in enumerate(PHASES)}
    per["total"] = float(sum(per.values()))
    print(json.dumps({"waves": int(len(live)), "ticks_per_tile": {k: round(v, 1) for k, v in per.items()}}))


if __name__ == "__main__":
    main()
