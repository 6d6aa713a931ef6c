"""Training on MI355X -- drop-in for the reference's src/ml/train.py.

Same public names, CLI flags, checkpoint keys and output files as the
reference (src/ml/train.py:35-385). What changes is underneath
VAETrainer.train_epoch / validate: for a DataLoader over a
UserInteractionDataset the whole epoch runs in the fused, graph-captured
HIP step of hvae/executor.py over the device-resident CSR (no per-row
densification, no host copy, no per-batch sync). Any other iterable of dense
batches is accepted too (each batch goes through the same fused step).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import pickle
import time
from pathlib import Path

import numpy as np
import pandas as pd
import torch
from scipy.sparse import csr_matrix
from torch.utils.data import DataLoader, Dataset, RandomSampler

from hvae import io as hio
from hvae import ops
from hvae.dist import init_from_env, is_main
from hvae.executor import AnnealedBeta, ConstBeta, DeviceData, FusedTrainer

from ..config import config
from ..preprocessing.embeddings import load_embeddings
from .model import HybridVAE, create_hybrid_vae, vae_loss_function  # noqa: F401  (re-exported API)

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger(__name__)


# =============================================================================
# Dataset
# =============================================================================


class UserInteractionDataset(Dataset):
    """Dataset of user interaction rows (reference: train.py:35-47).

    Indexing densifies a row (reference behaviour, used by generic loaders);
    VAETrainer instead reads the CSR it holds directly on the device.
    """

    def __init__(self, interaction_matrix: csr_matrix, user_indices: list[int] | None = None):
        self.interaction_matrix = interaction_matrix
        self.user_indices = user_indices or list(range(interaction_matrix.shape[0]))
        self._device_cache: dict = {}

    def __len__(self) -> int:
        return len(self.user_indices)

    def __getitem__(self, idx: int) -> torch.Tensor:
        user_vector = self.interaction_matrix[self.user_indices[idx]].toarray().flatten()
        return torch.FloatTensor(user_vector)

    def device_data(self, device: torch.device) -> DeviceData:
        key = str(device)
        if key not in self._device_cache:
            self._device_cache[key] = DeviceData.from_scipy(self.interaction_matrix, self.user_indices, device)
        return self._device_cache[key]


# =============================================================================
# Optimizer view (torch.optim.Adam-compatible state_dict over the fused state)
# =============================================================================


class HipAdam(torch.optim.Optimizer):
    """torch.optim.Adam semantics on the fused flat state of a FusedTrainer.

    ``state_dict()`` has torch.optim.Adam's layout (per-param step/exp_avg/
    exp_avg_sq, same param_groups keys), so checkpoints look like the
    reference's. ``step()`` applies Adam to externally computed ``.grad``
    tensors (module-API use); VAETrainer never calls it -- its epochs run the
    fused step, which includes clip + Adam.
    """

    def __init__(self, params, fused: FusedTrainer, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=False)
        super().__init__(params, defaults)
        self.fused = fused
        lay = fused.layout
        self._moments = {}
        for name, p in fused.param_views.items():
            if name == "encoder.0.weight":
                m, v = fused.m_w1t.t(), fused.v_w1t.t()
            else:
                m, v = lay.view(fused.m, name), lay.view(fused.v, name)
            self._moments[p] = (m, v)

    def _sync_state(self):
        self.fused.flush()
        step = float(self.fused.step_dev.item())
        for p, (m, v) in self._moments.items():
            if step > 0:
                self.state[p] = {"step": torch.tensor(step), "exp_avg": m, "exp_avg_sq": v}

    def state_dict(self):
        self._sync_state()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        """torch.optim.Adam.load_state_dict, then the loaded moments and step count become the fused state
        (m, v copied into the flat buffers, step_dev set, every W1t row marked current at that step) and the
        loaded hyper-parameters the fused step's (resume: reference src/ml/evaluate.py:273-291 loads the same
        checkpoint dict)."""
        super().load_state_dict(state_dict)
        self.fused.flush()  # rows behind the current step catch up before their moments are replaced
        step = None
        for p, (m, v) in self._moments.items():
            st = self.state.get(p)
            if not st:
                continue
            m.copy_(st["exp_avg"])
            v.copy_(st["exp_avg_sq"])
            step = int(float(st["step"]))
            self.state[p] = {"step": torch.tensor(float(step)), "exp_avg": m, "exp_avg_sq": v}
        if step is not None:
            self.fused.step_dev.fill_(step)
            self.fused.host_step = step
            self.fused._check_steps(0)
        self.fused.mark_all_current()
        self.sync_hyper()

    def sync_hyper(self):
        """param_groups[0]'s lr / betas / eps / weight_decay -> the fused step (an LR scheduler's change is seen
        by the next epoch; captured graphs are keyed on these values and re-captured)."""
        g0 = self.param_groups[0]
        f = self.fused
        f.lr, f.betas, f.eps, f.wd = float(g0["lr"]), tuple(float(b) for b in g0["betas"]), float(g0["eps"]), \
            float(g0["weight_decay"])

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        g0 = self.param_groups[0]
        cfg = ops.adam_config(g0["lr"], g0["betas"], g0["eps"], g0["weight_decay"], self.fused.step_dev, None)
        self.fused.flush()  # W1t rows current before the dense update of every row
        for p, (m, v) in self._moments.items():
            if p.grad is None:
                continue
            g = torch.empty_like(p)
            g.copy_(p.grad)
            ops.adam_dense(cfg, p, m, v, g)  # p, m, v, g share one dense memory order
        ops.counter_add(self.fused.step_dev, 1)
        self.fused.mark_all_current()
        return loss


class ModuleAdam(torch.optim.Optimizer):
    """torch.optim.Adam on the module's own parameter tensors, applied by libhvae (hvae_adam_dense), with the
    reference's clip_grad_norm_(max_norm) folded in (hvae_clip_grad_norm over the concatenated gradients, its
    coefficient applied inside the Adam kernel). Used by VAETrainer when the item embeddings are trainable
    (HybridVAE(freeze_embeddings=False), reference model.py:72-75): E is then a [N, d] parameter with a dense
    gradient, which the fused step's layout does not hold. state_dict() has torch.optim.Adam's layout."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=False)
        super().__init__(params, defaults)
        plist = [p for g in self.param_groups for p in g["params"]]
        dev = plist[0].device
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        self.norm = torch.zeros(1, device=dev)
        self.coef = torch.ones(1, device=dev)
        for p in plist:
            self.state[p] = {"step": torch.tensor(0.0), "exp_avg": torch.zeros_like(p),
                             "exp_avg_sq": torch.zeros_like(p)}

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        steps = [int(float(st["step"])) for st in self.state.values() if "step" in st]
        if steps:
            self.step_dev.fill_(steps[0])

    @torch.no_grad()
    def step(self, closure=None, max_norm: float | None = None):
        """One Adam step on every parameter with a gradient; max_norm: clip the global gradient norm first
        (torch.nn.utils.clip_grad_norm_ semantics, train.py:96)."""
        loss = closure() if closure is not None else None
        params = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
        if not params:
            return loss
        g0 = self.param_groups[0]
        coef = None
        if max_norm is not None:
            flat = torch.cat([p.grad.reshape(-1) for p in params])
            ops.clip_grad_norm(flat, None, max_norm, self.norm, self.coef)
            coef = self.coef
        cfg = ops.adam_config(g0["lr"], g0["betas"], g0["eps"], g0["weight_decay"], self.step_dev, coef)
        for p in params:
            st = self.state[p]
            g = torch.empty_like(p)  # p's memory order (W1 is an item-major view): p, m, v, g elementwise aligned
            g.copy_(p.grad)
            ops.adam_dense(cfg, p, st["exp_avg"], st["exp_avg_sq"], g)
        ops.counter_add(self.step_dev, 1)
        t = float(self.step_dev.item())
        for p in params:
            self.state[p]["step"] = torch.tensor(t)
        return loss


# =============================================================================
# Trainer
# =============================================================================


class VAETrainer:
    """Trainer for HybridVAE (reference: train.py:55-145)."""

    def __init__(self, model: HybridVAE, device: torch.device, lr: float = 0.001, weight_decay: float = 0.0,
                 precision: str | None = None, process_group=None):
        """process_group: user-batch data parallelism over its ranks (hvae/dist.py): every rank holds the
        whole dataset and takes its slice of each global batch of batch_size x world users."""
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.model = model.to(device)
        self.device = device
        if getattr(model, "item_embeddings_trainable", False) and (
                process_group is not None or os.environ.get("HVAE_TRAINABLE_E_MODULE", "0") == "1"):
            # trainable E under data parallelism (or HVAE_TRAINABLE_E_MODULE=1): the module-API step on libhvae
            # kernels (scores materialised per batch, as the reference does), E updated with the other parameters
            if process_group is not None:
                raise NotImplementedError("data parallelism covers frozen item embeddings only")
            self.fused = None
            self.optimizer = ModuleAdam(model.parameters(), lr=lr, weight_decay=weight_decay)
        else:
            self.fused = FusedTrainer(self.model, device, lr=lr, weight_decay=weight_decay,
                                      precision=precision or (config.PRECISION or None), process_group=process_group)
            self.optimizer = HipAdam(model.parameters(), self.fused, lr=lr, weight_decay=weight_decay)
        self.train_losses: list[float] = []
        self.val_losses: list[float] = []
        self.train_recon_losses: list[float] = []
        self.train_kl_losses: list[float] = []
        logger.info(f"Trainer on {device}, {sum(p.numel() for p in model.parameters()):,} params, "
                    f"decoder {self.fused.precision if self.fused is not None else 'module path (trainable E)'}"
                    f"{' (trainable E)' if getattr(model, 'item_embeddings_trainable', False) and self.fused else ''}")

    # beta of one training batch (reference: _compute_loss, train.py:71-79): AnnealedVAE's schedule runs on the
    # device inside the captured step (AnnealedBeta), so annealed epochs replay one graph like constant-beta ones
    def _beta_fn(self):
        m = self.model
        if hasattr(m, "compute_loss"):
            return AnnealedBeta(m)
        return ConstBeta(m.beta)

    def _run_module(self, loader, train: bool) -> dict[str, float]:
        """Reference train_epoch / validate (train.py:81-124) on the module API: dense batches, forward, loss,
        backward, clip 5.0, Adam -- every op a libhvae kernel."""
        tot = np.zeros(3)
        n = 0
        for batch in loader:
            x = batch.to(self.device).float()
            if train:
                self.optimizer.zero_grad()
                recon_x, mu, logvar = self.model(x)
                if hasattr(self.model, "compute_loss"):
                    loss, recon, kl = self.model.compute_loss(recon_x, x, mu, logvar)
                    self.model.step_annealing()
                else:
                    loss, recon, kl = vae_loss_function(recon_x, x, mu, logvar, self.model.beta)
                loss.backward()
                self.optimizer.step(max_norm=5.0)
            else:
                with torch.no_grad():
                    recon_x, mu, logvar = self.model(x)
                    loss, recon, kl = vae_loss_function(recon_x, x, mu, logvar, self.model.beta)
            tot += np.array([loss.item(), recon.item(), kl.item()])
            n += 1
        return {"total_loss": float(tot[0] / n), "recon_loss": float(tot[1] / n), "kl_loss": float(tot[2] / n)}

    def _run(self, loader, train: bool) -> dict[str, float]:
        if self.fused is None:
            return self._run_module(loader, train)
        self.optimizer.sync_hyper()
        p_drop = float(self.model.dropout)
        beta_fn = self._beta_fn() if train else ConstBeta(self.model.beta)
        ds = getattr(loader, "dataset", None)
        if isinstance(loader, DataLoader) and isinstance(ds, UserInteractionDataset):
            shuffle = isinstance(loader.sampler, RandomSampler)
            gen = getattr(loader.sampler, "generator", None) if shuffle else None
            data = ds.device_data(self.device)
            data.dp_global = self.fused.dp is not None  # every rank has every user; ranks slice global batches
            return self.fused.run_epoch(data, loader.batch_size, shuffle, beta_fn, p_drop,
                                        train=train, drop_last=loader.drop_last, generator=gen)
        # generic iterable of dense [B, N] batches
        tot = np.zeros(3)
        n = 0
        for i, batch in enumerate(loader):
            x = batch.to(self.device)
            csr = ops.dense_to_csr(x)
            data = DeviceData(csr.row_ptr, csr.col_idx, csr.vals, users=None, n_items=x.shape[1],
                              row_nnz=np.zeros(0, np.int64))
            loss3 = self.fused.step_batch(data, None, x.shape[0], beta_fn(i), p_drop, train=train)
            tot += np.array(loss3.tolist())
            n += 1
        return {"total_loss": float(tot[0] / n), "recon_loss": float(tot[1] / n), "kl_loss": float(tot[2] / n)}

    def train_epoch(self, loader) -> dict[str, float]:
        self.model.train()
        return self._run(loader, True)

    def validate(self, loader) -> dict[str, float]:
        self.model.eval()
        with torch.no_grad():
            return self._run(loader, False)

    def save_checkpoint(self, path: str | Path, epoch: int, is_best: bool = False, extra: dict | None = None) -> None:
        checkpoint = {
            "epoch": epoch,
            "model_state_dict": self.model.state_dict(),
            "optimizer_state_dict": self.optimizer.state_dict(),
            "train_losses": self.train_losses,
            "val_losses": self.val_losses,
            "train_recon_losses": self.train_recon_losses,
            "train_kl_losses": self.train_kl_losses,
            **(extra or {}),
        }
        torch.save(checkpoint, path)
        if is_best:
            best_path = Path(path).parent / "best_model.pth"
            torch.save(checkpoint, best_path)
            logger.info(f"Saved best model to {best_path}")


# =============================================================================
# Data Loading (reference: train.py:153-193)
# =============================================================================


def load_training_data(data_dir: str) -> tuple[csr_matrix, pd.DataFrame, pd.DataFrame, dict]:
    path = Path(data_dir)
    with open(path / "interaction_matrix.pkl", "rb") as f:
        matrix = pickle.load(f)  # the project's own dataset artifact (src/preprocessing/dataset.py)
    train_df = pd.read_csv(path / "train.csv", low_memory=False)
    val_df = pd.read_csv(path / "val.csv", low_memory=False)
    with open(path / "mappings.pkl", "rb") as f:
        mappings = pickle.load(f)
    logger.info(f"Loaded: matrix {matrix.shape}, train {len(train_df)}, val {len(val_df)}")
    return matrix, train_df, val_df, mappings


def get_user_indices_from_df(df: pd.DataFrame, user_to_idx: dict[str, int]) -> list[int]:
    return [user_to_idx[uid] for uid in df["user_id"].unique() if uid in user_to_idx]


def _build_matrix(df: pd.DataFrame, user_to_idx: dict, item_to_idx: dict, shape: tuple) -> csr_matrix:
    """Positives (binary_rating == 1) with duplicate pairs summed (reference: train.py:175-182)."""
    positives = df[df["binary_rating"] == 1] if "binary_rating" in df.columns else df
    rows = positives["user_id"].map(user_to_idx)
    cols = positives["asin"].map(item_to_idx)
    return csr_matrix((np.ones(len(positives)), (rows, cols)), shape=shape)


def _get_device(device: str | None = None) -> torch.device:
    if device:
        dev = torch.device(device)
        if dev.type != "cuda":  # the reference's cpu / mps choices parse, then fail here, before any data loads
            raise RuntimeError(f"device {device!r}: the MI355X HybridVAE path runs on a HIP device only; "
                               "there is no CPU fallback.")
        return dev
    if torch.cuda.is_available():
        return torch.device("cuda")
    raise RuntimeError("The MI355X HybridVAE path needs a HIP device (torch.cuda on ROCm); none is visible. "
                       "There is no CPU fallback.")


# =============================================================================
# Main Training Function (reference: train.py:201-342)
# =============================================================================


def train_hybrid_vae(
    data_dir: str,
    embeddings_path: str,
    output_dir: str,
    latent_dim: int = 200,
    hidden_dims: list[int] | None = None,
    batch_size: int = 512,
    epochs: int = 100,
    learning_rate: float = 0.001,
    weight_decay: float = 0.0,
    beta: float = 0.2,
    dropout: float = 0.5,
    use_annealing: bool = False,
    patience: int = 10,
    device: str | None = None,
    ignore_embeddings: bool = False,
    precision: str | None = None,
) -> None:
    # under torchrun (WORLD_SIZE > 1): one process per GPU, user-batch data parallel over RCCL; batch_size is
    # per GPU (the global batch is batch_size x world) and only rank 0 writes checkpoints and the history
    group = init_from_env() if (device is None or str(device).startswith("cuda")) else None
    main_rank = is_main(group)
    dev = _get_device(device)
    logger.info(f"Using device: {dev}" + (f" (rank {torch.distributed.get_rank()} of "
                                           f"{torch.distributed.get_world_size()})" if group is not None else ""))
    output_path = Path(output_dir)
    if main_rank:
        output_path.mkdir(parents=True, exist_ok=True)

    # load_training_data + _build_matrix + get_user_indices_from_df in one native pass per file (hvae/io.py);
    # the matrices and user lists are those of the reference's pandas path (tests/test_io_cpu.py)
    t_load = time.perf_counter()
    shape, train_matrix, val_matrix, train_users, val_users, mappings = hio.load_training_csr(data_dir)
    n_items = shape[1]
    logger.info(f"Loaded: matrix {shape}, train {train_matrix.nnz} / val {val_matrix.nnz} positives "
                f"({time.perf_counter() - t_load:.2f} s)")

    emb_path = Path(embeddings_path)
    mappings_path = emb_path.with_name(f"{emb_path.stem}_mappings.pkl")
    embeddings, emb_item_to_idx, _ = load_embeddings(embeddings_path, str(mappings_path))
    assert emb_item_to_idx and len(emb_item_to_idx) == n_items, (
        f"Embedding mismatch: {len(emb_item_to_idx) if emb_item_to_idx else 0} vs {n_items}")
    if ignore_embeddings:
        logger.info("Using random embeddings instead of SBERT")
        embeddings = np.random.normal(0, 0.01, embeddings.shape).astype(np.float32)

    train_loader = DataLoader(UserInteractionDataset(train_matrix, train_users),
                              batch_size=batch_size, shuffle=True, num_workers=0)
    val_loader = DataLoader(UserInteractionDataset(val_matrix, val_users),
                            batch_size=batch_size, shuffle=False, num_workers=0)

    # the reference's len(train_loader) * epochs * 0.5 counts optimizer steps; under data parallelism one step covers
    # batch_size x world users, so the schedule counts the global steps (ceil(n / (B W)) per epoch), and the
    # annealed beta of step s is the single-GPU value at batch size B W
    world = torch.distributed.get_world_size(group) if group is not None else 1
    steps_per_epoch = -(-len(train_users) // (batch_size * world)) if world > 1 else len(train_loader)
    anneal_steps = int(steps_per_epoch * epochs * 0.5)
    model = create_hybrid_vae(n_items=n_items, item_embeddings=embeddings, latent_dim=latent_dim,
                              hidden_dims=hidden_dims, dropout=dropout, beta=beta, use_annealing=use_annealing,
                              anneal_steps=anneal_steps)
    logger.info(f"Model: {sum(p.numel() for p in model.parameters()):,} params")

    trainer = VAETrainer(model, dev, learning_rate, weight_decay, precision=precision, process_group=group)
    best_val_loss, patience_counter = float("inf"), 0
    start_time = time.time()
    for epoch in range(epochs):
        logger.info(f"\nEpoch {epoch + 1}/{epochs}")
        train_metrics = trainer.train_epoch(train_loader)
        val_metrics = trainer.validate(val_loader)
        trainer.train_losses.append(train_metrics["total_loss"])
        trainer.val_losses.append(val_metrics["total_loss"])
        trainer.train_recon_losses.append(train_metrics["recon_loss"])
        trainer.train_kl_losses.append(train_metrics["kl_loss"])
        logger.info(f"Train: {train_metrics['total_loss']:.4f} (recon={train_metrics['recon_loss']:.4f}, "
                    f"kl={train_metrics['kl_loss']:.4f})")
        logger.info(f"Val: {val_metrics['total_loss']:.4f}")
        is_best = val_metrics["total_loss"] < best_val_loss
        if is_best:
            best_val_loss = val_metrics["total_loss"]
            patience_counter = 0
        else:
            patience_counter += 1
        if main_rank:  # replicas are bit-identical: one writer
            trainer.save_checkpoint(
                output_path / f"checkpoint_epoch_{epoch + 1}.pth", epoch + 1, is_best,
                extra={"train_metrics": train_metrics, "val_metrics": val_metrics,
                       "model_config": {"n_items": n_items, "latent_dim": latent_dim, "hidden_dims": hidden_dims,
                                        "beta": beta, "dropout": dropout}})
        if patience_counter >= patience:
            logger.info(f"Early stopping at epoch {epoch + 1}")
            break

    training_time = time.time() - start_time
    if main_rank:
        with open(output_path / "training_history.json", "w") as f:
            json.dump({"train_losses": trainer.train_losses, "val_losses": trainer.val_losses,
                       "train_recon_losses": trainer.train_recon_losses, "train_kl_losses": trainer.train_kl_losses,
                       "training_time_seconds": round(training_time, 2)}, f, indent=2)
    logger.info(f"Training complete! Best val loss: {best_val_loss:.4f}")
    logger.info(f"Total training time: {training_time:.1f}s")


def main() -> None:
    parser = argparse.ArgumentParser(description="Train Hybrid VAE (MI355X)")
    parser.add_argument("--data", default=str(config.DATA_DIR))
    parser.add_argument("--embeddings", default=config.EMBEDDINGS_FILE)
    parser.add_argument("--output", default=str(config.MODEL_DIR))
    parser.add_argument("--latent-dim", type=int, default=config.LATENT_DIM)
    parser.add_argument("--hidden-dims", type=int, nargs="+", default=[config.HIDDEN_DIM])
    parser.add_argument("--batch-size", type=int, default=config.BATCH_SIZE)
    parser.add_argument("--epochs", type=int, default=config.EPOCHS)
    parser.add_argument("--learning-rate", type=float, default=config.LEARNING_RATE)
    parser.add_argument("--weight-decay", type=float, default=0.0)
    parser.add_argument("--beta", type=float, default=0.2)
    parser.add_argument("--dropout", type=float, default=0.5)
    parser.add_argument("--use-annealing", action="store_true")
    parser.add_argument("--patience", type=int, default=20)
    parser.add_argument("--device", choices=["cuda", "cpu", "mps"])
    parser.add_argument("--ignore-embeddings", action="store_true")
    parser.add_argument("--precision", choices=["bf16", "fp8", "fp32"], default=None,
                        help="decoder MFMA precision (default: bf16 where a kernel exists)")
    args = parser.parse_args()
    train_hybrid_vae(data_dir=args.data, embeddings_path=args.embeddings, output_dir=args.output,
                     latent_dim=args.latent_dim, hidden_dims=args.hidden_dims, batch_size=args.batch_size,
                     epochs=args.epochs, learning_rate=args.learning_rate, weight_decay=args.weight_decay,
                     beta=args.beta, dropout=args.dropout, use_annealing=args.use_annealing, patience=args.patience,
                     device=args.device, ignore_embeddings=args.ignore_embeddings, precision=args.precision)
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
