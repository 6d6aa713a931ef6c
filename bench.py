#!/usr/bin/env python3
"""HybridVAE train throughput (users/sec) on MI355X -- the BASELINE.json metric.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload syn10m|syn1m|all_beauty|appliances]

One "step" = one fused train step (encoder -> reparam/KL -> projection ->
streaming decoder + multinomial loss -> backward -> clip 5.0 -> Adam) over
one batch of users of a synthetic interaction matrix shaped like the named
workload. Default: the north-star config (BASELINE.json configs[3]) on one
GPU -- a 1.25 M-user shard (10 M users / 8 GPUs) of the 10M x 1M synthetic,
d = 768, latent 128, hidden [512], 4096 users per GPU per step, bf16 decoder
MFMA. Inputs (CSR, weights, frozen E) are resident in HBM before the timed
region. N > 1 runs one process per GPU (torchrun), user-batch data parallel
with the gradient exchange over RCCL (weak scaling: B users per GPU per step;
--scaling strong splits a fixed --global-batch over the GPUs).

Prints ONE JSON line on rank 0, with a live roofline for the dominant kernel
(HIP events around its launches on the stream it runs on) and the CPU
oracle (oracle/ref_cpu.py, a pinned restatement of the reference trainer)
timed on this host's cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "recommendation-system_amd"), str(ROOT), str(ROOT / "tests" / "golden")]

import torch  # noqa: E402

WORKLOADS = {
    # BASELINE.json configs[1]: All_Beauty (22,363 x 12,101, d=384, latent=128), best config hidden [512],
    # dropout 0.3, beta 0.2, lr 1e-3, batch 64 (config.BATCH_SIZE used by `make train-best`)
    "all_beauty": dict(users=22363, items=12101, d=384, latent=128, hidden=[512], batch=64, lam=3.0,
                       dropout=0.3, beta=0.2, lr=1e-3),
    # configs[0]: Appliances (2,072 x 890, d=384, latent=64)
    "appliances": dict(users=2072, items=890, d=384, latent=64, hidden=[512], batch=64, lam=3.0,
                       dropout=0.3, beta=0.2, lr=1e-3),
    # configs[2]: synthetic 1M users x 100K items, d=384, batch 4096 (hidden [512], latent 128)
    "syn1m": dict(users=1_000_000, items=100_000, d=384, latent=128, hidden=[512], batch=4096, lam=15.0,
                  dropout=0.3, beta=0.2, lr=1e-3),
    # configs[3]: synthetic 10M users x 1M items, d=768, batch 4096 per GPU. Each rank generates only its
    # own 10M / 8 users (a dense 10M-row matrix per rank would not fit host memory 8 times over); the CPU
    # baseline runs B = 256 (the dense B x N batch of the reference loader is 16 GB at 4096)
    "syn10m": dict(users=10_000_000, items=1_000_000, d=768, latent=128, hidden=[512], batch=4096, lam=15.0,
                   dropout=0.3, beta=0.2, lr=1e-3, shard_gen=True, cpu_batch=256),
}

PEAK_HBM_GBS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md, spec)
PEAK_BF16_TFLOPS = 2500.0  # dense bf16 MFMA
PEAK_FP8_TFLOPS = 5000.0   # dense fp8 (block-scaled e4m3) MFMA
PEAK_F32_TFLOPS = 157.3    # f32 MFMA = f32 vector rate
# L2-served fills into LDS with every CU streaming: 16.8-18.8 TB/s (MI355X_MICROARCH.md, 'Indexed rows: gather into
# LDS', rows shared by every workgroup); the upper end, so a fraction against it is not flattering
PEAK_L2_LDS_GBS = 18800.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_data(w: dict, rank: int, world: int):
    from gen import synth_csr, synth_embeddings
    E = synth_embeddings(w["items"], w["d"], seed=1)
    if w.get("shard_gen"):  # this rank's users only (a 1/8 shard: the 8-GPU split), from a per-rank seed
        X = synth_csr(w["users"] // 8, w["items"], lam=w["lam"], seed=1000 + rank)
        return X, E, np.arange(X.shape[0])
    X = synth_csr(w["users"], w["items"], lam=w["lam"], seed=0)
    return X, E, np.arange(X.shape[0])  # every rank holds every user and takes its slice of each global batch


def batch_stats(X, users, B: int, gen_seed: int = 0, samples: int = 32) -> tuple[float, float]:
    """Mean distinct items (W1t rows with a gradient) and mean stored entries of a batch of B users."""
    rng = np.random.default_rng(gen_seed)
    tot = nnz = 0
    for _ in range(samples):
        rows = rng.choice(users, size=min(B, len(users)), replace=False)
        sub = X[rows]
        tot += len(np.unique(sub.indices))
        nnz += sub.nnz
    return tot / samples, nnz / samples


def host_cores() -> tuple[int, str]:
    """CPUs this process may run on (affinity, capped by a cgroup CPU quota) and the CPU model."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:  # cgroup v2 quota ("max 100000" = unlimited)
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            n = max(1, min(n, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, model


def cpu_baseline(w: dict, X, E, seconds: float, threads: int | None = None) -> dict:
    """The pinned CPU restatement of the reference trainer on this host's cores.

    Per batch: the reference loader's per-row densification (UserInteractionDataset
    .__getitem__ + collate, src/ml/train.py:45-47) then one train step
    (fwd, loss, backward, clip 5.0, Adam; src/ml/train.py:81-103) -- the work of
    one GPU step -- run by oracle.ref_cpu.CpuTrainer: the reference's own module
    layout (nn.Linear / LayerNorm / GELU / Dropout, F.log_softmax, clip_grad_norm_,
    torch.optim.Adam), pinned to the golden steps like the oracle
    (tests/test_oracle_golden.py::test_cpu_trainer_steps). BASELINE.md's 8-thread
    calibration of the reference (All_Beauty, B = 64: 1,836 users/s step-only) is
    not reproducible to +-10 % in the build container: back-to-back runs of the
    same step there take 50-160 ms (shared host), so the baseline is reported, not
    asserted. The loader and the step are timed separately: "value" is the
    two in series (the reference's num_workers=0 DataLoader), "step_only" the
    step alone.
    """
    from oracle import ref_cpu as R
    cores, model = host_cores()
    threads = threads or cores
    torch.set_num_threads(threads)
    B = w.get("cpu_batch", w["batch"])
    p = R.init_params(w["items"], E, w["latent"], w["hidden"], seed=0)
    trainer = R.CpuTrainer(p, w["dropout"], lr=w["lr"])  # the reference's modules, Adam, clip_grad_norm_
    rng = np.random.default_rng(0)
    order = rng.permutation(X.shape[0])
    t_load = t_step = 0.0

    def one(i, timed):
        nonlocal t_load, t_step
        t0 = time.perf_counter()
        rows = order[(i * B) % (len(order) - B):][:B]
        x = torch.stack([torch.FloatTensor(X[int(u)].toarray().flatten()) for u in rows])
        t1 = time.perf_counter()
        trainer.step(x, w["beta"])  # dropout and the reparameterisation noise drawn as the reference draws them
        t2 = time.perf_counter()
        if timed:
            t_load += t1 - t0
            t_step += t2 - t1

    warm = 3  # 3 warm-up steps, then >= 20 steps or >= 60 s
    for i in range(warm):
        one(i, False)
    n, t0 = 0, time.perf_counter()
    while True:
        one(n + warm, True)
        n += 1
        el = time.perf_counter() - t0
        if n >= 20 or el >= seconds:
            break
    return {"value": round(n * B / (t_load + t_step), 2), "unit": "users/s", "cores": threads, "kind": "port",
            "step_only": round(n * B / t_step, 2), "loader_only": round(n * B / t_load, 2),
            "cpu_model": model, "host_cpus_usable": cores,
            "sample": f"{warm} warm-up + {n} timed steps x {B} users of the same synthetic workload (per-row "
                      f"densifying loader + fwd/bwd/clip/Adam in series), {el:.1f} s timed, torch fp32 on {threads} "
                      f"CPU threads"}


# kernel families the library's probe can bracket (ProbeScope names in csrc/)
FAMILIES = ("decoder_sweep", "decoder_finalize", "gemm", "adam_rows", "adam_catchup", "adam_pending", "encoder_fwd",
            "ln_bwd", "rowgrad_plan", "rowgrad_apply", "clip", "mlp_fwd", "mlp_bwd")


def roofline_models(w: dict, precision: str, B: int, fused, X, users, rank: int, kernels: dict) -> dict:
    """Algorithmic work per launch and the bound each family is measured against.

    decoder_sweep: 4 B N D flop (S = U E^T and O = P E; no dE, E is frozen), MFMA-bound when those flops take
      longer at peak than reading E once (2 B, 1 B or 4 B per element) takes at 8 TB/s, HBM-bound otherwise.
    gemm: the exact-fp32 MFMA GEMMs of the step: heads, projection forward, and their data and weight
      gradients, 6 B (2 L H + d L + d^2) flop per step, split evenly over the launches per step.
    adam_rows (lazy exact Adam): p, m, v (24 B per element) of the batch's unique W1t rows and of the 1/period of
      W1t rows the rotating g = 0 sweep brings up to date (plus 8 B per swept row), and p, m, v, g (28 B) of
      the small dense parameters; with HVAE_DENSE_ADAM=1 all N rows.
    encoder_fwd: the gathered W1t rows (nnz H 4 B) + h, xhat (B H 8 B) written.
    decoder_finalize: split partials read (splits B (D + 2) 4 B), the batch's fp32 E rows (nnz D 4 B), dU written.
    """
    N, H, D, Lt = w["items"], w["hidden"][0], w["d"], w["latent"]
    uniq, nnz = batch_stats(X, users, B, gen_seed=rank)
    out = {}

    def put(name, bound, alg, peak, unit, **extra):
        t, n = kernels[name]
        if t <= 0 or n <= 0:
            return
        ach = alg / t / (1e12 if unit == "TFLOP/s" else 1e9)
        out[name] = {"bound": bound, "achieved": ach, "peak": peak, "unit": unit, "alg_per_launch": alg,
                     "avg_launch_us": t * 1e6, **extra}

    dec_flops = 4.0 * B * N * D
    dec_bytes = {"bf16": 2.0, "fp8": 1.0, "fp32": 4.0}[precision] * N * D + 8.0 * B * D
    dec_peak = {"bf16": PEAK_BF16_TFLOPS, "fp8": PEAK_FP8_TFLOPS, "fp32": PEAK_F32_TFLOPS}[precision]
    # the second bound of the sweep: every user block streams the whole image from L2 into LDS (the users that
    # share an E tile: hvae_decoder_users_per_tile), against the L2-served LDS-fill rate
    from hvae import _lib as L
    upt = int(L.lib().hvae_decoder_users_per_tile({"bf16": L.HVAE_BF16, "fp8": L.HVAE_FP8, "fp32": L.HVAE_F32}[precision],
                                                  B, N, D))
    img = {"bf16": 2.0, "fp8": 1.0, "fp32": 4.0}[precision] * N * D
    t_dec = kernels["decoder_sweep"][0]
    l2 = None
    if upt > 0 and t_dec > 0:
        l2b = -(-B // upt) * img
        l2 = {"bound": "l2_lds", "users_per_tile": upt, "bytes_per_launch": l2b, "achieved": l2b / t_dec / 1e9,
              "peak": PEAK_L2_LDS_GBS, "unit": "GB/s", "frac": round(l2b / t_dec / 1e9 / PEAK_L2_LDS_GBS, 4)}
    if dec_flops / (dec_peak * 1e12) >= dec_bytes / (PEAK_HBM_GBS * 1e9):
        put("decoder_sweep", "mfma", dec_flops, dec_peak, "TFLOP/s", l2_lds=l2)
    else:
        put("decoder_sweep", "hbm", dec_bytes, PEAK_HBM_GBS, "GB/s", l2_lds=l2,
            tflops=round(dec_flops / t_dec / 1e12, 3) if t_dec else None)
    n_gemm = max(kernels["gemm"][1], 1)
    # batches <= 1024 run the latent / projection forward and data gradients in the row-parallel MLP launches
    # (hvae_mlp_*_rows); their GEMM launches are the weight gradients only (one third of the flops)
    rows = fused._mlp_rows_ok(B)
    gemm_flops = (2.0 if rows else 6.0) * B * (2 * Lt * H + (D * Lt + D * D if Lt != D else 0))
    for k in range(1, len(w["hidden"])):
        gemm_flops += 6.0 * B * w["hidden"][k] * w["hidden"][k - 1]
    put("gemm", "mfma", gemm_flops / n_gemm, PEAK_F32_TFLOPS, "TFLOP/s")
    n_small = fused.layout.n_small
    if fused.lazy_adam and fused._defers(B):
        # deferred update (hvae_adam_lazy_defer): the launch steps the dense segment and only records the gradient
        # rows (item_of read; pend item / slot and last_step written: 16 B a row); their bytes move to the next
        # step's catch-up and hvae_adam_lazy_pending ("adam_pending", timed in launch_us, no model: how many of the
        # rows the catch-up takes first depends on the next batch)
        adam_bytes = 16.0 * uniq + 28.0 * n_small
    elif fused.lazy_adam:
        from hvae._lib import lib
        swept = -(-N // int(lib().hvae_adam_lazy_sweep_period(N)))
        adam_bytes = 24.0 * H * (uniq + swept) + 8.0 * swept + 28.0 * n_small
    else:
        adam_bytes = 24.0 * N * H + 4.0 * N + 28.0 * n_small
    put("adam_rows", "hbm", adam_bytes, PEAK_HBM_GBS, "GB/s")
    put("encoder_fwd", "hbm", 4.0 * nnz * H + 8.0 * B * H, PEAK_HBM_GBS, "GB/s")
    if rows:
        # every block streams the three weight matrices once (from L2): blocks x weight bytes, + the encoder's
        # gathered W1t rows in the forward launch when it runs there (one hidden layer)
        R = 1 if B <= 32 else 2 if B <= 512 else 4
        wbytes = 4.0 * (2 * Lt * H + D * Lt + D * D) * -(-B // R)
        enc = 4.0 * nnz * H if len(w["hidden"]) == 1 and H <= 512 else 0.0
        put("mlp_fwd", "l2", wbytes + enc, PEAK_L2_LDS_GBS, "GB/s")
        put("mlp_bwd", "l2", wbytes, PEAK_L2_LDS_GBS, "GB/s")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--workload", default="syn10m", choices=sorted(WORKLOADS))
    ap.add_argument("--batch-size", type=int, default=None)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp8", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=60.0,
                    help="CPU baseline: time >= 20 steps or this many seconds, whichever comes first (SURVEY §8d)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--probe-steps", type=int, default=50)
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --batch-size users per GPU per step (default); strong: --global-batch users per "
                         "step split over the GPUs (SURVEY §8d: both curves)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling: users per step over all GPUs (default: the workload's batch)")
    args = ap.parse_args()

    w = dict(WORKLOADS[args.workload])
    if args.batch_size:
        w["batch"] = args.batch_size
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.scaling == "strong":
        G = args.global_batch or w["batch"]
        if G % world:
            raise SystemExit(f"--global-batch {G} is not divisible by {world} GPUs")
        w["batch"] = G // world
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(torch.cuda.device_count(), 1)
    local = local % ndev  # more ranks than GPUs (a 1-GPU rehearsal with HVAE_DIST_BACKEND=gloo) share devices
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    group = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("HVAE_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
        group = dist.group.WORLD

    from hvae.executor import ConstBeta, FusedTrainer
    from src.ml.model import HybridVAE

    X, E, users = make_data(w, rank, world)
    torch.manual_seed(0)
    model = HybridVAE(w["items"], E, latent_dim=w["latent"], hidden_dims=w["hidden"], dropout=w["dropout"],
                      beta=w["beta"]).to(device)
    fused = FusedTrainer(model, device, lr=w["lr"], precision=args.precision, seed=1234, use_graphs=True,
                         process_group=group)
    data = fused.device_data(X, users)
    data.dp_global = world > 1 and not w.get("shard_gen")  # per-rank generated shards are already disjoint
    B = w["batch"]
    n_per_epoch = len(users) // (B * (world if data.dp_global else 1))
    beta = ConstBeta(w["beta"])
    gen = torch.Generator(device=device).manual_seed(rank)  # epoch orders drawn on the GPU

    def run(nsteps):
        done = 0
        while done < nsteps:
            k = min(nsteps - done, n_per_epoch)
            fused.run_epoch(data, B, True, beta, w["dropout"], generator=gen, max_batches=k)
            done += k

    run(args.warmup)
    # the wall time is never taken from probed steps: an armed probe puts a 200-us hold kernel in front of every
    # bracketed launch (csrc/hvae_abi.hip, probe_mark), so the library is disarmed here and armed only after the
    # timed region, for the separate probe pass below
    from hvae._lib import check as _check, lib as _lib
    _check(_lib().hvae_probe_arm(None, 0), "probe_disarm")
    if group is not None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if group is not None:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if group is not None:
        on_dev = torch.distributed.get_backend(group) == "nccl"
        t = torch.tensor([elapsed], device=device if on_dev else "cpu", dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed

    # ---- live per-kernel timing: libhvae brackets each launch of the armed kernel family with a hipEvent pair
    # recorded on the stream it runs on (eager steps of the same workload, after the timed region)
    import ctypes as C
    from hvae._lib import check, lib
    from hvae.provenance import kernel_source_digest
    N, H, D, Lt = w["items"], w["hidden"][0], w["d"], w["latent"]
    fused.use_graphs = False

    def probe(name):
        check(lib().hvae_probe_arm(name.encode(), 64 * args.probe_steps), "probe_arm")
        run(args.probe_steps)
        torch.cuda.synchronize()
        avg, n = C.c_double(), C.c_int()
        check(lib().hvae_probe_collect(C.byref(avg), C.byref(n)), "probe_collect")
        check(lib().hvae_probe_arm(None, 0), "probe_disarm")
        return avg.value * 1e-6, n.value // args.probe_steps

    kernels = {name: probe(name) for name in FAMILIES}
    fused.use_graphs = True
    roof = roofline_models(w, args.precision, B, fused, X, users, rank, kernels)
    # the dominant kernel family: the largest per-step total (average launch x launches per step) among the
    # families with an algorithmic model (the row-parallel MLP launches against the L2-served rate their weight
    # streams are read at)
    dom = max((k for k in roof if roof[k]["peak"]), key=lambda k: kernels[k][0] * max(kernels[k][1], 1))
    r = roof[dom]
    traffic, stale = None, None
    pmc = ROOT / "profiles" / (f"pmc_{args.workload}.json" if args.precision == "bf16"
                               else f"pmc_{args.workload}_{args.precision}.json")
    if pmc.exists():
        try:
            doc = json.loads(pmc.read_text())
            if doc.get("src_sha") == kernel_source_digest():
                traffic = doc.get(dom, {}).get("hbm_bytes_per_launch")
            else:  # measured on other kernel sources: refuse it
                stale = {"pmc_src_sha": doc.get("src_sha"), "tree_src_sha": kernel_source_digest()}
        except (ValueError, OSError):
            traffic = None
    roofline = {"bound": r["bound"], "achieved": round(r["achieved"], 2), "peak": r["peak"], "unit": r["unit"],
                "frac": round(r["achieved"] / r["peak"], 4), "traffic": traffic, "kernel": dom,
                "avg_launch_us": round(r["avg_launch_us"], 2),
                "alg_per_launch": r["alg_per_launch"]}
    if r.get("l2_lds"):  # the sweep's second bound: L2 -> LDS bytes of its user blocks
        roofline["l2_lds"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r["l2_lds"].items()}
    if stale:
        roofline["traffic_stale"] = stale
    launch_us = {k: {"avg_us": round(v[0] * 1e6, 2), "launches_per_step": v[1],
                     "us_per_step": round(v[0] * 1e6 * v[1], 2)} for k, v in kernels.items()}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(w, X, E, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": "HybridVAE train users/sec",
            "value": round(value, 1),
            "unit": "users/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (Zipf(0.8) items, 5+Poisson rows, L2-normalised random E; random-init weights)",
            "config": {"workload": args.workload, "users": w["users"], "users_resident": int(len(users)),
                       "items": w["items"], "emb_dim": D,
                       "latent": w["latent"], "hidden": w["hidden"], "global_batch": B * world,
                       "batch_per_gpu": B, "parallelism": f"dp{world}", "decoder": args.precision},
            "roofline": roofline,
            "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in roof.items()},
            "src_sha": kernel_source_digest(),
            "launch_us": launch_us,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if group is not None:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
