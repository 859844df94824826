"""Shared test setup: markers, import paths, tolerances.

-m "not gpu": oracle vs golden vectors, host logic, C-ABI exports (no device).
-m gpu:       parity of the HIP path against the CPU oracle, through the C-ABI.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kaldi-fp16_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running")


def rel_fro(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (den if den > 0 else 1.0))


def max_abs_rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    m = np.max(np.abs(b))
    return float(np.max(np.abs(a - b)) / (m if m > 0 else 1.0))


@pytest.fixture(scope="session")
def gpu():
    """Initialise device 0 through the bridge ABI; skip cleanly without a GPU."""
    import kfp16
    if kfp16.core.bridge_gpu_init(0) != 0:
        pytest.skip("no GPU: " + (kfp16.core.bridge_last_error() or b"").decode())
    return kfp16
