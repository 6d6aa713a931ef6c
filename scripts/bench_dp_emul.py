"""One rank's data-parallel step at W ranks, emulated on ONE GPU.

    python scripts/bench_dp_emul.py [--world 8] [--steps 20] [--warmup 6] [--workload syn10m] [--precision bf16|fp8]

The step of rank 0 of a W-rank job is the single-GPU step over its own batch of B users plus the work the
exchange adds: the union batch's row-gradient plan (beside the forward), its apply over the gathered da, the
clip over the union's rows and lazy Adam over every union row (hvae/dist.py). Here the collectives are replaced
by local copies: the other W - 1 ranks' CSR packets are real batches of B users drawn from W - 1 other
synthetic shards (same generator, other seeds), packed with hvae_csr_batch_pack exactly as those ranks would,
and their da are fixed random [B, H] blocks. Everything after the copies is the product code path
(FusedTrainer._run_epoch_dp with its three captured graphs), so the timed steps contain every kernel a rank
runs. What it cannot contain is the wire time of the two all-gathers; it is estimated from the bytes per step
(reported, not added). Prints one JSON line per world size measured (W = 1 is the plain single-GPU path).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "recommendation-system_amd"), str(ROOT), str(ROOT / "tests" / "golden")]

import torch  # noqa: E402

from bench import WORKLOADS, make_data  # noqa: E402


MARKS = []  # (tag, host time, device event) while ARMED
ARMED = [False]


def mark(tag):
    """A step-phase boundary: the host clock and a hipEvent on the current stream (every phase of a rank's step
    is enqueued on it in order: the three graphs and the exchanges between them)."""
    if ARMED[0]:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        MARKS.append((tag, time.perf_counter(), e))


def phase_report(marks):
    """Median per-step phase times from the marks of the timed run: device (event to event) and host (enqueue
    clock), plus what lies outside the steps (the epoch's host setup and its closing sync)."""
    steps, cur = [], None
    for tag, ht, ev in marks:
        if tag == "s":
            cur = {"s": (ht, ev)}
            steps.append(cur)
        elif cur is not None:
            cur[tag] = (ht, ev)
    full = [st for st in steps if "e" in st]
    if len(full) < 3:
        return {}
    order = [t for t in ("s", "csr0", "csr1", "g0", "g1", "e") if t in full[0]]
    names = {("s", "csr0"): "pre_graph", ("csr0", "csr1"): "csr_exchange", ("csr1", "g0"): "main_graph",
             ("g0", "g1"): "grad_exchange", ("g1", "e"): "update_graph", ("s", "e"): "step_graphs"}
    out = {"device_ms": {}, "host_ms": {}}
    body = full[1:-1]  # steady state: drop the first and the last step of the run
    for a, b in zip(order, order[1:]):
        nm = names.get((a, b), f"{a}-{b}")
        out["device_ms"][nm] = round(float(np.median([st[a][1].elapsed_time(st[b][1]) for st in body])), 4)
        out["host_ms"][nm] = round(float(np.median([(st[b][0] - st[a][0]) * 1e3 for st in body])), 4)
    nxt = list(zip(full, full[1:]))[1:]
    out["device_ms"]["step_to_step"] = round(float(np.median([a["s"][1].elapsed_time(b["s"][1]) for a, b in nxt])), 4)
    out["host_ms"]["step_to_step"] = round(float(np.median([(b["s"][0] - a["s"][0]) * 1e3 for a, b in nxt])), 4)
    out["steps_marked"] = len(full)
    out["run_span_ms"] = round((full[-1]["e"][0] - full[0]["s"][0]) * 1e3, 3)
    return out


def make_emul_exchange(world, device, n_items, H, n_small, packets_fn):
    """A DPExchange whose rank-0 collectives are served from pre-packed packets of W - 1 synthetic ranks."""
    from hvae import dist as D

    class EmulExchange(D.DPExchange):
        def __init__(self):  # DPExchange.__init__ without a process group
            self.group, self.world, self.rank, self.device, self.backend = None, world, 0, device, "emul"
            self.n_items, self.H, self.ns = n_items, H, n_small
            self.pack_fn, self.merge_fn, self.make_merged = D._hip_pack, D._hip_merge, D._hip_make_merged
            self.B = self.cap = 0
            self.overflow = torch.zeros(1, dtype=torch.int32, device=device)
            self._plans, self._merged = {}, {}
            self.step_i = 0
            self.da_other = None

        def all_reduce(self, values, op=None):
            return np.asarray(values, dtype=np.float64)  # every emulated rank reports the same bookkeeping

        def communicate_csr(self):
            mark("csr0")
            pk = packets_fn(self.B, self.cap, self.L)  # [W - 1, batches, L] on the device
            self.recv_csr[0].copy_(self.send[self.ns:])
            self.recv_csr[1:].copy_(pk[:, self.step_i % pk.shape[1], self.ns:])
            mark("csr1")

        def communicate_grads(self):
            mark("g0")
            self.recv_g[0].copy_(self.send_g)
            self.recv_g[1:].copy_(self.send_g.expand(self.world - 1, -1))
            B = self.B
            self.recv_da[:B].copy_(self.send_da)
            if self.da_other is None or self.da_other.shape[0] != (self.world - 1) * B:
                g = torch.Generator(device=self.device).manual_seed(7)
                self.da_other = 1e-4 * torch.randn((self.world - 1) * B, self.H, generator=g, device=self.device)
            self.recv_da[B:].copy_(self.da_other)
            self.step_i += 1
            mark("g1")

    return EmulExchange()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="*", default=[1, 8])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--workload", default="syn10m", choices=sorted(WORKLOADS))
    ap.add_argument("--other-batches", type=int, default=8, help="distinct batches per emulated rank (cycled)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp8"])
    args = ap.parse_args()
    w = dict(WORKLOADS[args.workload])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from gen import synth_csr
    from hvae import _lib, ops
    from hvae._lib import check, lib, ptr
    from hvae.executor import ConstBeta, FusedTrainer
    from src.ml.model import HybridVAE

    X, E, users = make_data(w, 0, 1)
    B = w["batch"]
    H = w["hidden"][0]
    for W in args.world:
        torch.manual_seed(0)
        model = HybridVAE(w["items"], E, latent_dim=w["latent"], hidden_dims=w["hidden"], dropout=w["dropout"],
                          beta=w["beta"]).to(dev)
        fused = FusedTrainer(model, dev, lr=w["lr"], precision=args.precision, seed=1234,
                               use_graphs=True)
        replay0 = fused._replay

        def replay_marked(*a, **k):  # step boundaries for phase_report
            mark("s")
            n = replay0(*a, **k)
            mark("e")
            return n

        fused._replay = replay_marked
        data = fused.device_data(X, users)
        info = {}
        if W > 1:
            # the other ranks' batches: real CSR batches of B users from W - 1 other shards of the same generator
            others = []
            nb_o = args.other_batches
            for r in range(1, W):
                Xr = synth_csr(B * nb_o, w["items"], lam=w["lam"], seed=1000 + r)
                others.append(ops.csr_from_scipy(Xr, dev))
            own_cap = data.max_batch_nnz(B)
            other_cap = max(int((o.row_ptr[(k + 1) * B] - o.row_ptr[k * B]).item()) for o in others for k in range(nb_o))
            cap = max(own_cap, other_cap)
            cache = {}

            def packets_fn(Bq, capq, L):
                key = (Bq, capq)
                if key not in cache:
                    pk = torch.zeros(W - 1, nb_o, L, dtype=torch.float32, device=dev)
                    ns = fused.layout.n_small
                    for r, o in enumerate(others):
                        for k in range(nb_o):
                            rows = torch.arange(k * Bq, (k + 1) * Bq, dtype=torch.int32, device=dev)
                            x = _lib.CsrBatch(ptr(o.row_ptr), ptr(o.col_idx), ptr(o.vals), ptr(rows), None, Bq,
                                              w["items"])
                            flat = pk[r, k]
                            rp = flat[ns:ns + Bq + 1].view(torch.int32)
                            col = flat[ns + Bq + 1:ns + Bq + 1 + capq].view(torch.int32)
                            val = flat[ns + Bq + 1 + capq:]
                            check(lib().hvae_csr_batch_pack(C.byref(x), 1.0 / W, ptr(rp), ptr(col), ptr(val), capq,
                                                            ptr(fused.dp.overflow),
                                                            torch.cuda.current_stream(dev).cuda_stream), "pack")
                    torch.cuda.synchronize()
                    cache[key] = pk
                return cache[key]

            fused.dp = make_emul_exchange(W, dev, fused.layout.n_items, H, fused.layout.n_small, packets_fn)
            fused.dp_seed = 1234
            fused._dp_cap = lambda data_, B_: cap
            info = {"cap_per_rank": cap, "union_cap": W * cap}
        gen = torch.Generator(device=dev).manual_seed(0)
        n_per_epoch = len(users) // B
        beta = ConstBeta(w["beta"])

        def run(nsteps):
            done = 0
            while done < nsteps:
                k = min(nsteps - done, n_per_epoch)
                fused.run_epoch(data, B, True, beta, w["dropout"], generator=gen, max_batches=k)
                done += k

        run(args.warmup)
        torch.cuda.synchronize()
        MARKS.clear()
        ARMED[0] = True
        t0 = time.perf_counter()
        run(args.steps)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ARMED[0] = False
        info["phases"] = phase_report(MARKS)
        # (no "outside the steps" figure: run_span_ms is a host-timestamp span while the host runs ahead of the
        # device, so wall time minus it measures the host's lead, not device time outside the steps)
        if fused.dp is not None:
            fused.dp.check()
            info["union_unique_rows_last_step"] = int(fused.dp.merged.n_unique.item())
            # the bytes rank 0 receives per step through the two all-gathers (CSR packets, small gradients, da)
            L = fused.dp.L
            info["allgather_recv_bytes_per_step"] = int((W - 1) * (4 * (L - fused.layout.n_small) + 4 * fused.layout.n_small
                                                                 + 4 * B * H))
        out = {"probe": "dp_emul", "workload": args.workload, "precision": args.precision, "world": W, "B": B,
               "steps": args.steps,
               "ms_per_step": round(el / args.steps * 1e3, 4), **info}
        print(json.dumps(out), flush=True)
        del fused, model, data
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
