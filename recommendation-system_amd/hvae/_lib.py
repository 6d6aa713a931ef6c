"""ctypes binding of libhvae.so (the C ABI declared in include/hvae.h).

The shared library is built in-tree by ``make -C recommendation-system_amd lib``
(``hipcc --offload-arch=gfx950``). There is deliberately no fallback: if the
library is missing, or the tensors are not on a HIP device, every op raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("HVAE_LIB", _HERE / "libhvae.so"))

ABI_VERSION = 5  # include/hvae.h HVAE_ABI_VERSION
HVAE_OK = 0
HVAE_F32 = 0
HVAE_BF16 = 1
HVAE_FP8 = 2

EPI_NONE, EPI_BIAS, EPI_BIAS_GELU_DROP, EPI_GELU_DROP_BWD, EPI_DROP_BWD, EPI_REPARAM_BWD = range(6)

# Philox stream tags (csrc/hvae_common.h)
TAG_ENC_DROP = 0x100
TAG_PROJ_DROP = 0x200
TAG_EPS = 0x300

ROWSQ_PARTS = 16  # include/hvae.h HVAE_ROWSQ_PARTS

vp = C.c_void_p
i64 = C.c_int64
u64 = C.c_uint64
f32 = C.c_float
f64 = C.c_double
sz = C.c_size_t
cint = C.c_int
u32 = C.c_uint32


class CsrBatch(C.Structure):
    _fields_ = [("row_ptr", vp), ("col_idx", vp), ("vals", vp), ("rows", vp), ("rows_offset", vp), ("nb", i64),
                ("n_items", i64)]


class HostCsr(C.Structure):  # hvae_host_csr
    _fields_ = [("row_ptr", vp), ("col_idx", vp), ("vals", vp), ("n_rows", i64), ("n_cols", i64), ("nnz", i64),
                ("users", vp), ("n_users_seen", i64), ("n_records", i64)]


class RowGrad(C.Structure):
    _fields_ = [
        ("cnt", vp), ("slot_of", vp), ("item_of", vp), ("seg_off", vp), ("fill", vp),
        ("contrib_row", vp), ("contrib_val", vp), ("rows", vp), ("n_unique", vp),
        ("cap", i64), ("n_items", i64), ("contrib_slot", vp), ("part", vp), ("part_floats", i64), ("rowsq", vp),
    ]


class Epilogue(C.Structure):
    _fields_ = [
        ("kind", cint), ("bias", vp), ("pre_out", vp), ("pre_in", vp), ("p_drop", f32),
        ("drop_mult", vp), ("seed", u64), ("step_dev", vp), ("tag", u32), ("train", cint),
        ("opa_rowsum", vp), ("aux", vp), ("aux_scale", f32), ("aux_scale_dev", vp),
    ]


class GemmDesc(C.Structure):
    _fields_ = [
        ("trans_a", cint), ("trans_b", cint), ("M", i64), ("N", i64), ("K", i64), ("alpha", f32),
        ("A", vp), ("lda", i64), ("B", vp), ("ldb", i64), ("beta", f32), ("C", vp), ("ldc", i64),
        ("epi", C.POINTER(Epilogue)), ("ws", vp), ("ws_bytes", sz),
    ]


class MlpRows(C.Structure):  # hvae_mlp_rows
    _fields_ = [
        ("nb", i64), ("H", i64), ("L", i64), ("D", i64),
        ("W_heads", vp), ("b_heads", vp), ("W_a", vp), ("b_a", vp), ("W_b", vp), ("b_b", vp),
        ("train", cint), ("p_drop", f32), ("drop_mult", vp), ("eps_in", vp), ("seed", u64), ("step_dev", vp),
        ("h", vp), ("heads", vp), ("z", vp), ("eps", vp), ("kl_rows", vp), ("p1", vp), ("q", vp), ("u", vp),
        ("dU", vp), ("ks", f32), ("ks_dev", vp), ("dp1", vp), ("dheads", vp), ("dh", vp),
        ("plan_x", C.POINTER(CsrBatch)), ("plan_rg", C.POINTER(RowGrad)),
        ("ln_w", vp), ("ln_b", vp), ("xhat", vp), ("rstd", vp), ("enc_drop_mult", vp), ("enc_layer", u32),
        ("da", vp), ("d_ln_w", vp), ("d_ln_b", vp), ("d_bias", vp), ("ws", vp), ("ws_bytes", sz),
        ("enc_x", C.POINTER(CsrBatch)), ("w1t", vp), ("b1", vp),
        ("adam", C.c_void_p), ("adam_m", vp), ("adam_v", vp), ("last_step", vp), ("adam_tab", vp),
    ]


MLP_ROWS_MAX_NB = 1024  # include/hvae.h HVAE_MLP_ROWS_MAX_NB
PLAN_SMALL_CAP = 4096   # csrc/hvae_rgplan.h kPlanSmallCap (the one-block row-gradient plan)


class Adam(C.Structure):
    _fields_ = [
        ("lr", f64), ("beta1", f64), ("beta2", f64), ("eps", f64), ("weight_decay", f64),
        ("step_dev", vp), ("coef_dev", vp),
    ]


class AdamPend(C.Structure):  # hvae_adam_pend: a deferred W1t update's record (device pointers)
    _fields_ = [("slot_of", vp), ("item_of", vp), ("hdr", vp)]


P = C.POINTER
# name -> (restype, argtypes); mirrors include/hvae.h one to one.
SIGNATURES = {
    "hvae_version": (cint, []),
    "hvae_last_error": (cint, [C.c_char_p, sz]),
    "hvae_probe_arm": (cint, [C.c_char_p, cint]),
    "hvae_probe_collect": (cint, [C.POINTER(C.c_double), C.POINTER(cint)]),
    "hvae_dense_to_csr": (cint, [vp, i64, i64, vp, vp, vp, i64, vp, sz, vp]),
    "hvae_dense_to_csr_workspace": (sz, [i64, i64]),
    "hvae_encoder_fwd": (cint, [P(CsrBatch), vp, vp, vp, vp, i64, f32, vp, u64, vp, cint, vp, vp, vp, vp]),
    "hvae_ln_gelu_drop_fwd": (cint, [vp, vp, vp, i64, i64, f32, vp, u64, vp, u32, cint, vp, vp, vp, vp]),
    "hvae_ln_gelu_drop_bwd": (cint, [vp, vp, vp, vp, vp, i64, i64, f32, vp, u64, vp, u32, cint, vp, vp, vp,
                                     vp, vp, sz, vp]),
    "hvae_ln_gelu_drop_bwd_workspace": (sz, [i64, i64]),
    "hvae_w1_rowgrad": (cint, [P(CsrBatch), vp, i64, P(RowGrad), vp, sz, vp]),
    "hvae_w1_rowgrad_workspace": (sz, [i64]),
    "hvae_w1_rowgrad_plan": (cint, [P(CsrBatch), P(RowGrad), vp, sz, vp]),
    "hvae_w1_rowgrad_apply": (cint, [vp, i64, P(RowGrad), vp]),
    "hvae_rowgrad_to_dense": (cint, [P(RowGrad), i64, vp, i64, vp]),
    "hvae_csr_row_sums": (cint, [P(CsrBatch), vp, vp]),
    "hvae_softmax_weights": (cint, [vp, i64, i64, i64, vp, vp, f32, vp]),
    "hvae_rowgrad_scatter_rows": (cint, [P(RowGrad), i64, f32, vp, i64, vp]),
    "hvae_rowgrad_part_floats": (i64, [i64, i64]),
    "hvae_gemm_f32": (cint, [cint, cint, i64, i64, i64, f32, vp, i64, vp, i64, f32, vp, i64, P(Epilogue), vp,
                             sz, vp]),
    "hvae_gemm_f32_workspace": (sz, [i64, i64, i64]),
    "hvae_gemm_f32_pair": (cint, [P(GemmDesc), P(GemmDesc), vp]),
    "hvae_colsum": (cint, [vp, i64, i64, i64, f32, vp, vp, sz, vp]),
    "hvae_colsum_workspace": (sz, [i64, i64]),
    "hvae_reparam_kl_fwd": (cint, [vp, vp, i64, i64, i64, cint, vp, u64, vp, vp, vp, vp, vp]),
    "hvae_reparam_kl_bwd": (cint, [vp, vp, vp, i64, vp, i64, i64, f32, vp, cint, vp, vp, i64, vp]),
    "hvae_anneal_beta": (cint, [vp, f64, f64, i64, i64, vp, vp]),
    "hvae_mlp_fwd_rows": (cint, [P(MlpRows), vp]),
    "hvae_mlp_bwd_rows": (cint, [P(MlpRows), vp]),
    "hvae_mlp_bwd_rows_workspace": (sz, [i64, i64]),
    "hvae_mlp_rows_blocks": (i64, [i64]),
    "hvae_mlp_rows_supported": (cint, [i64, i64, i64, i64, cint]),
    "hvae_gemm_f32_multi": (cint, [P(GemmDesc), cint, vp]),
    "hvae_decoder_image_bytes": (sz, [cint, i64, i64]),
    "hvae_decoder_image": (cint, [cint, vp, i64, i64, vp, vp]),
    "hvae_decoder_fwd": (cint, [cint, vp, i64, vp, vp, i64, i64, i64, vp, vp, vp, sz, vp]),
    "hvae_decoder_workspace": (sz, [cint, i64, i64, i64]),
    "hvae_decoder_users_per_tile": (i64, [cint, i64, i64, i64]),
    "hvae_decoder_supported": (cint, [cint, i64]),
    "hvae_row_norm_max": (cint, [cint, vp, i64, i64, vp, vp]),
    "hvae_decoder_bwd": (cint, [P(CsrBatch), vp, i64, vp, i64, vp, vp, f32, vp, vp, vp]),
    "hvae_decoder_train": (cint, [cint, vp, i64, vp, vp, vp, P(CsrBatch), i64, f32, vp, vp, vp, vp, vp, f32, vp,
                                  vp, vp, vp, sz, vp]),
    "hvae_nll_rows_fwd": (cint, [vp, i64, vp, i64, i64, i64, vp, vp, vp]),
    "hvae_nll_rows_bwd": (cint, [vp, i64, vp, i64, vp, i64, i64, f32, vp, i64, vp]),
    "hvae_loss_finalize": (cint, [vp, vp, i64, f32, vp, vp, vp]),
    "hvae_clip_grad_norm": (cint, [vp, i64, P(RowGrad), i64, f32, vp, vp, vp, sz, vp]),
    "hvae_clip_grad_norm_step": (cint, [vp, i64, P(RowGrad), i64, f32, vp, vp, vp, vp, vp, i64, vp, sz, vp]),
    "hvae_clip_grad_norm_workspace": (sz, [i64, i64, i64]),
    "hvae_adam_dense": (cint, [P(Adam), vp, vp, vp, vp, i64, vp]),
    "hvae_adam_rows": (cint, [P(Adam), vp, vp, vp, P(RowGrad), i64, i64, vp]),
    "hvae_adam_flat": (cint, [P(Adam), vp, vp, vp, P(RowGrad), i64, i64, vp, i64, i64, vp]),
    "hvae_clip_grad_norm_step_adam": (cint, [vp, i64, P(RowGrad), i64, f32, vp, vp, vp, vp, vp, i64, P(Adam), vp,
                                             vp, sz, vp]),
    "hvae_adam_lazy": (cint, [P(Adam), vp, i64, vp, vp, vp, vp, P(RowGrad), i64, vp, i64, i64, vp]),
    "hvae_adam_lazy_catchup": (cint, [P(Adam), vp, vp, vp, vp, vp, P(RowGrad), i64, i64, vp]),
    "hvae_adam_lazy_catchup_csr": (cint, [P(Adam), vp, vp, vp, vp, vp, P(CsrBatch), i64, vp]),
    "hvae_adam_lazy_sweep_period": (cint, [i64]),
    "hvae_adam_lazy_defer": (cint, [P(Adam), vp, i64, vp, vp, vp, vp, P(RowGrad), i64, vp, i64, i64, P(AdamPend),
                                    vp]),
    "hvae_adam_lazy_catchup_csr_pending": (cint, [P(Adam), vp, vp, vp, vp, vp, P(CsrBatch), i64, P(AdamPend), vp]),
    "hvae_adam_lazy_pending": (cint, [P(Adam), vp, vp, vp, vp, vp, i64, i64, i64, P(AdamPend), vp]),
    "hvae_counter_add": (cint, [vp, i64, vp]),
    "hvae_counters_add": (cint, [vp, i64, vp, i64, vp]),
    "hvae_score_candidates": (cint, [vp, i64, vp, vp, i64, vp, i64, i64, vp, vp]),
    "hvae_rank_first": (cint, [vp, i64, i64, vp, vp]),
    "hvae_topk": (cint, [vp, i64, i64, i64, P(CsrBatch), i64, vp, vp, vp]),
    "hvae_topk_fused_workspace": (sz, [i64, i64, i64, i64]),
    "hvae_topk_fused": (cint, [vp, i64, vp, vp, vp, i64, i64, P(CsrBatch), i64, i64, vp, vp, vp, vp, sz,
                               vp]),
    "hvae_cast_bf16": (cint, [vp, vp, i64, vp]),
    "hvae_negatives_legacy": (cint, [vp, vp, vp, i64, vp, i64, vp, vp, i64, C.c_int32, vp, vp]),
    "hvae_read_interactions": (cint, [C.c_char_p, C.c_char_p, i64, i64, C.c_char_p, i64, i64, cint,
                                      P(HostCsr)]),
    "hvae_host_csr_free": (None, [P(HostCsr)]),
    "hvae_csr_batch_pack": (cint, [P(CsrBatch), f32, vp, vp, vp, i64, vp, vp]),
}

_lib = None


def lib() -> C.CDLL:
    """Load libhvae.so once (after torch, so the HIP runtime torch loaded is reused)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"libhvae.so not found at {LIB_PATH}; build it with "
                f"`make -C {LIB_PATH.parent.parent} lib` (hipcc --offload-arch=gfx950). "
                "There is no CPU fallback for the HybridVAE MI355X path."
            )
        L = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.hvae_version() != ABI_VERSION:
            raise RuntimeError(f"libhvae ABI version {L.hvae_version()} != {ABI_VERSION}")
        _lib = L
    return _lib


def last_error() -> str:
    buf = C.create_string_buffer(1024)
    lib().hvae_last_error(buf, 1024)
    return buf.value.decode(errors="replace")


def check(rc: int, what: str) -> None:
    if rc != HVAE_OK:
        raise RuntimeError(f"{what} failed (rc={rc}): {last_error()}")


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def require_hip(*ts: torch.Tensor | None) -> None:
    for t in ts:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError(
                "HybridVAE MI355X path: tensors must live on the HIP device (torch 'cuda' on ROCm); "
                f"got {t.device}. There is no CPU fallback."
            )
