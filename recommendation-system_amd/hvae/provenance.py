"""Provenance stamps for committed measurements.

A PMC summary (profiles/pmc_<workload>.json) is only valid for the kernel
sources it was measured on. kernel_source_digest() hashes every file the
library is built from; scripts/pmc_to_traffic.py stamps it into the summary
and bench.py reports the summary's traffic only when the stamp matches the
tree it runs from.
"""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG = Path(__file__).resolve().parents[1]
ROOT = PKG.parent


def kernel_source_files() -> list[Path]:
    files = sorted((PKG / "csrc").glob("*.hip")) + sorted((PKG / "csrc").glob("*.h"))
    files.append(ROOT / "include" / "hvae.h")
    return files


def kernel_source_digest() -> str:
    h = hashlib.sha256()
    for f in kernel_source_files():
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]
