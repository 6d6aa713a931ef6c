import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "recommendation-system_amd"
# repo root (oracle/, tests/golden) and the drop-in package (src.ml.*, hvae)
for p in (str(ROOT), str(PKG), str(ROOT / "tests" / "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libhvae.so")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return dict(np.load(ROOT / "tests" / "golden" / "golden.npz", allow_pickle=False))


@pytest.fixture(scope="session")
def golden_meta():
    import json
    return json.loads((ROOT / "tests" / "golden" / "golden_meta.json").read_text())


@pytest.fixture(scope="session")
def hip_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)
