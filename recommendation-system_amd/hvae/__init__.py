"""hvae -- MI355X-native runtime of the HybridVAE train/eval path.

libhvae.so (csrc/, C ABI in include/hvae.h) holds the HIP kernels; this package
binds it (``_lib``), wraps it for torch tensors (``ops``), provides the autograd
functions of the module API (``autograd``), the fused graph-captured train-step
executor (``executor``) and the data-parallel exchange (``dist``).
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
