"""Data-parallel fused training on the GPU: two ranks sharing cuda:0 over gloo (a one-GPU rehearsal of the
RCCL path -- the same executor code, collectives staged through host memory).

  * a 2-rank step over batches of B users equals a 1-rank step over their union of 2B users (dropout masks
    and reparameterisation noise injected, the union's slices on each rank): losses, every parameter and both
    Adam moments, up to the order of the dense reductions (the first-layer row gradient of the union is
    rebuilt from the gathered (x, da) by the same kernels, in the union's batch order);
  * replicas stay bit-identical through graph-captured epochs, over pre-sharded equal data and over the
    shared-permutation sharding of the drop-in trainer (uneven last batch: one rank may have no users), and
    they learn.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        _worker_body(rank, world, port, q)
    except BaseException:  # surface the rank's error in the parent's output before the queue breaks
        import traceback
        traceback.print_exc()
        raise


def _worker_body(rank, world, port, q):
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(150, exit=False)  # a stuck rank names where it waits
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "recommendation-system_amd"), str(root), str(root / "tests" / "golden")]
    import torch.distributed as dist
    from gen import synth_csr, synth_embeddings
    from hvae.executor import ConstBeta, FusedTrainer
    from src.ml.model import HybridVAE
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    X = synth_csr(600, 900, seed=21)
    E = synth_embeddings(900, 128, seed=22)
    torch.manual_seed(0)
    model = HybridVAE(900, E, latent_dim=64, hidden_dims=[128], dropout=0.3, beta=0.2).to(dev)
    fused = FusedTrainer(model, dev, precision="bf16", seed=5, use_graphs=True, process_group=dist.group.WORLD)
    data = fused.device_data(X, list(range(rank, 600, world)))
    gen = torch.Generator().manual_seed(100 + rank)
    losses = [fused.run_epoch(data, 32, True, ConstBeta(0.2), 0.3, generator=gen)["total_loss"] for _ in range(3)]
    # validation over per-rank shards: every rank validates its whole shard and the batch losses are summed over
    # the ranks; compared below with each shard's own single-rank validation, batch-weighted
    val = fused.run_epoch(data, 32, False, ConstBeta(0.2), 0.3, train=False)
    dp_saved, fused.dp = fused.dp, None
    val_local = fused.run_epoch(data, 32, False, ConstBeta(0.2), 0.3, train=False)
    fused.dp = dp_saved
    torch.cuda.synchronize()
    # numpy arrays pickle by value: a torch CPU tensor would travel as a shared-memory fd, which the parent can
    # only open while this process is alive (it may already have exited: EOFError in the parent)
    q.put((rank, losses, fused.flat.cpu().numpy(), fused.m.cpu().numpy(), fused.v.cpu().numpy(),
           int(fused.step_dev.item()), (val, val_local, (len(range(rank, 600, world)) + 31) // 32)))
    dist.barrier()
    dist.destroy_process_group()


def _step_worker(rank, world, port, q, cfg=None):
    try:
        _step_body(rank, world, port, q, cfg)
    except BaseException:
        import traceback
        traceback.print_exc()
        raise


# (n_users, n_items, d, L, H, B per rank, lam, decoder precision): the small shape, and the Syn-1M shape (B = 4096
# per rank, 100 K items) whose union of two ranks (> 150 K entries) takes the sorted row-gradient plan
# (hvae_rgsort.hip) of the product build
SMALL = (200, 700, 384, 64, [256], 24, 5.0, "fp32")
SYN1M = (8192, 100_000, 384, 128, [512], 4096, 15.0, "fp32")


def _step_body(rank, world, port, q, cfg=None):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "recommendation-system_amd"), str(root), str(root / "tests" / "golden")]
    import numpy as np
    import torch.distributed as dist
    from gen import synth_csr, synth_embeddings
    from hvae.executor import FusedTrainer
    from src.ml.model import HybridVAE
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n_users, n_items, d, L, Hd, B, lam, prec = cfg or SMALL
    p = 0.3
    X = synth_csr(n_users, n_items, lam=lam, seed=31)
    E = synth_embeddings(n_items, d, seed=32)
    g = torch.Generator().manual_seed(33)
    union = torch.randperm(n_users, generator=g)[: world * B].int()
    enc = (torch.rand(world * B, Hd[0], generator=g) >= p).float() / (1 - p)
    proj = (torch.rand(world * B, d, generator=g) >= p).float() / (1 - p)
    eps = torch.randn(world * B, L, generator=g)

    def run(group, rows, sl):
        from hvae import ops
        torch.manual_seed(0)
        model = HybridVAE(n_items, E, latent_dim=L, hidden_dims=Hd, dropout=p, beta=0.2).to(dev)
        # fp32 decoder: the bf16 sweep's P rounding depends on its item-split plan, which depends on the batch
        # size (B vs 2B), a 1e-3 effect that would hide the exchange's own exactness
        fused = FusedTrainer(model, dev, precision=prec, seed=3, use_graphs=False, process_group=group)
        data = fused.device_data(X, list(range(n_users)))
        ext = {"enc_masks": [enc[sl].to(dev)], "proj_mask": proj[sl].to(dev), "eps": eps[sl].to(dev)}
        losses = [fused.step_batch(data, rows.to(dev), len(rows), 0.2, p, train=True, ext=ext).cpu().numpy()]
        # step 1's gradients (what clip + Adam consume): the small dense ones, the first layer's rows, the norm
        rg = fused.dp.merged if fused.dp is not None else fused._bufs[(len(rows), True)].rg
        w1 = torch.zeros(n_items, Hd[0], device=dev)
        ops.rowgrad_to_dense(rg, w1)
        extra = {}
        if fused.dp is not None:
            # the union's row gradient against float64 sum_r w_r X_r^T da_r, independent of either plan
            da = fused._bufs[(len(rows), True)].da[0].cpu()
            das = [torch.empty_like(da) for _ in range(world)]
            dist.all_gather(das, da, group=group)
            want = torch.zeros(n_items, Hd[0], dtype=torch.float64, device=dev)
            for r_ in range(world):
                sub = X[union[r_ * B:(r_ + 1) * B].numpy()].tocoo()
                Xr = torch.zeros(B, n_items, dtype=torch.float64, device=dev)  # densified on the device
                Xr.index_put_((torch.as_tensor(sub.row, device=dev).long(), torch.as_tensor(sub.col, device=dev).long()),
                              torch.as_tensor(sub.data, dtype=torch.float64, device=dev), accumulate=True)
                want += (1.0 / world) * (Xr.t() @ das[r_].to(dev).double())
                del Xr
            extra["rowgrad_rel"] = float((w1.double() - want).abs().max() / want.abs().max())
            extra["uniq"] = int(rg.n_unique.item())
            extra["cap"] = int(rg.struct.cap)
        grads = (fused.g_small.cpu().numpy(), w1.cpu().numpy() if n_items * Hd[0] <= 10 ** 6 else None,
                 float(fused.norm.item()), extra)
        losses.append(fused.step_batch(data, rows.to(dev), len(rows), 0.2, p, train=True, ext=ext).cpu().numpy())
        torch.cuda.synchronize()
        flat = fused.flat.cpu().numpy()
        if n_items * Hd[0] > 10 ** 6:  # large: the parameters as a digest of max-abs and checksum slices
            flat = flat[-200_000:]
        return losses, grads, flat

    mine = slice(rank * B, (rank + 1) * B)
    dp = run(dist.group.WORLD, union[mine], mine)
    ref = run(None, union, slice(0, world * B)) if rank == 0 else None
    q.put((rank, dp, ref))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [SMALL, SYN1M], ids=["small", "syn1m_sorted_plan"])
def test_dp_step_equals_union_step(hip_device, cfg):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_step_worker, args=(r, world, port, q, cfg)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (_, (l0, g0, f0), ref), (_, (l1, g1, f1), _) = res
    lr_, gr, fr = ref
    assert (f0 == f1).all()  # replicas identical
    import numpy as np
    for s in range(2):  # the union batch's loss = mean of the two equal shares
        np.testing.assert_allclose((l0[s] + l1[s]) / 2, lr_[s], rtol=2e-5, atol=1e-6)
    rel = lambda a, b: float(np.abs(a.astype(np.float64) - b).max() / max(np.abs(b).max(), 1e-30))
    # step 1's gradients: equal up to the order of the dense reductions over users (B + B vs 2B); the first
    # layer's row gradient is rebuilt from the gathered (x, da) in the union's batch order
    assert rel(g0[0], gr[0]) < 2e-5, rel(g0[0], gr[0])
    if g0[1] is not None:
        assert rel(g0[1], gr[1]) < 2e-5, rel(g0[1], gr[1])
    assert abs(g0[2] - gr[2]) <= 2e-5 * gr[2]
    assert g0[3]["rowgrad_rel"] < 1e-5, g0[3]  # the union's row gradient = float64 sum_r w_r X_r^T da_r
    if cfg is SYN1M:
        assert g0[3]["cap"] >= 150_000, g0[3]  # the product build's sorted plan (kSortedPlanMinCap)
    # parameters after two Adam steps: Adam turns a near-zero gradient's sign into a +-lr step, so compare
    # within 2 lr per step of each other
    assert float(np.abs(f0.astype(np.float64) - fr).max()) <= 2 * 2 * 1e-3 * (1 + 1e-3)


def _global_worker(rank, world, port, q):
    try:
        import sys
        from pathlib import Path
        root = Path(__file__).resolve().parents[1]
        sys.path[:0] = [str(root / "recommendation-system_amd"), str(root), str(root / "tests" / "golden")]
        import torch.distributed as dist
        from gen import synth_csr, synth_embeddings
        from hvae.executor import ConstBeta, FusedTrainer
        from src.ml.model import HybridVAE
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        X = synth_csr(417, 900, seed=41)  # 417 = 6 x (2 x 32) + 33: a last global batch of 17 + 16
        E = synth_embeddings(900, 128, seed=42)
        torch.manual_seed(0)
        model = HybridVAE(900, E, latent_dim=64, hidden_dims=[128], dropout=0.3, beta=0.2).to(dev)
        fused = FusedTrainer(model, dev, precision="bf16", seed=5, use_graphs=True, process_group=dist.group.WORLD)
        data = fused.device_data(X, list(range(417)))
        data.dp_global = True
        r = [fused.run_epoch(data, 32, True, ConstBeta(0.2), 0.3) for _ in range(3)]
        # shuffled sharded validation: the order comes from the shared seed, so both ranks deal the same batches
        r.append(fused.run_epoch(data, 32, True, ConstBeta(0.2), 0.3, train=False))
        # with a caller's generator (seeded differently per rank) the order is rank 0's draw, broadcast
        gen = torch.Generator().manual_seed(100 + rank)
        r.append(fused.run_epoch(data, 32, True, ConstBeta(0.2), 0.3, train=False, generator=gen))
        # ... and the caller's generator ends where a single-GPU validation leaves it
        from hvae.executor import _sampler_order
        ref = torch.Generator().manual_seed(100 + rank)
        _sampler_order(417, ref, dev)
        r.append(bool(torch.equal(gen.get_state(), ref.get_state())))
        torch.cuda.synchronize()
        q.put((rank, r, fused.flat.cpu().numpy(), int(fused.step_dev.item())))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        traceback.print_exc()
        raise


def test_dp_global_sharding_epochs(hip_device):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_global_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (_, ra, fa, sa), (_, rb, fb, sb) = res
    assert sa == sb == 3 * 7  # 6 full global batches + the partial one, per epoch
    assert ra == rb  # the union losses, all-reduced (and the shuffled validation, dealt from the shared seed)
    assert (fa == fb).all()
    assert ra[2]["total_loss"] < ra[0]["total_loss"]
    assert all(abs(v) < float("inf") for v in ra[3].values())
    assert all(abs(v) < float("inf") for v in ra[4].values())
    assert ra[5] is True and rb[5] is True


def _defer_worker(rank, world, port, q):
    """Data-parallel epochs with the deferred W1t update against the undeferred one, in one process group: the
    union's pending rows are moved by the next step's catch-up (this rank's batch) and hvae_adam_lazy_pending (the
    rest), and the last global batch (385 = 6 x 64 + 1: one user on rank 0, none on rank 1) resolves them eagerly
    on the empty rank."""
    try:
        import sys
        from pathlib import Path
        root = Path(__file__).resolve().parents[1]
        sys.path[:0] = [str(root / "recommendation-system_amd"), str(root), str(root / "tests" / "golden")]
        import torch.distributed as dist
        from gen import synth_csr, synth_embeddings
        from hvae.executor import ConstBeta, FusedTrainer
        from src.ml.model import HybridVAE
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        X = synth_csr(385, 900, seed=51)
        E = synth_embeddings(900, 128, seed=52)
        out = []
        for defer in ("0", "1"):
            os.environ["HVAE_ADAM_DEFER"] = defer
            torch.manual_seed(0)
            model = HybridVAE(900, E, latent_dim=64, hidden_dims=[128], dropout=0.3, beta=0.2).to(dev)
            fused = FusedTrainer(model, dev, precision="bf16", seed=5, use_graphs=True,
                                 process_group=dist.group.WORLD)
            assert fused._defers(32) == (defer == "1")
            data = fused.device_data(X, list(range(385)))
            data.dp_global = True
            r = [fused.run_epoch(data, 32, True, ConstBeta(0.2), 0.3) for _ in range(2)]
            torch.cuda.synchronize()
            out.append((r, fused.flat.cpu().numpy(), fused.m.cpu().numpy(), fused.v.cpu().numpy()))
        (ra, fa, ma, va), (rb, fb, mb, vb) = out
        q.put((rank, ra == rb, bool((fa == fb).all() and (ma == mb).all() and (va == vb).all())))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        traceback.print_exc()
        raise


def test_dp_deferred_adam_is_bitwise(hip_device):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_defer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(r[1] and r[2] for r in res), res


def test_dp_two_ranks_one_gpu(hip_device):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (_, la, fa, ma, va, sa, vla), (_, lb, fb, mb, vb, sb, vlb) = [
        (r, l_, torch.from_numpy(f), torch.from_numpy(m), torch.from_numpy(v), s_, vl)
        for r, l_, f, m, v, s_, vl in res]
    assert sa == sb == 3 * ((300 + 31) // 32)
    assert torch.equal(fa, fb) and torch.equal(ma, mb) and torch.equal(va, vb)  # replicas identical
    assert torch.isfinite(fa).all()
    assert la[-1] < la[0] and lb[-1] < lb[0]
    # validation on per-rank shards: both ranks report the batch-weighted mean over both shards' batches
    (val_a, loc_a, na), (val_b, loc_b, nb) = vla, vlb
    for key in ("total_loss", "recon_loss", "kl_loss"):
        assert val_a[key] == val_b[key]
        want = (loc_a[key] * na + loc_b[key] * nb) / (na + nb)
        assert abs(val_a[key] - want) <= 1e-9 * abs(want), (key, val_a[key], want)
