import os
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "gpu-radix-sort_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: long-running (large sizes)")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    return oracle


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    g = json.loads((ROOT / "tests" / "golden" / "pcg_golden.json").read_text())
    v = np.load(ROOT / "tests" / "golden" / "vectors.npz")
    return g, v
