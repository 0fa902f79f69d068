"""pytest configuration: markers, import paths and golden-fixture helpers.

`-m "not gpu"` runs on any CPU box; `-m gpu` needs a HIP device and the
in-tree libyolo_hip.so (build with `make` or __graft_entry__.build()).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "yolo-infer-pt_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device and the built libyolo_hip.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    path = os.path.join(GOLD, name)
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)
