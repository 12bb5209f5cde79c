import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dstd-gcn_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def load_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def group(d, prefix):
    """Sub-dict of an npz keyed '<prefix>/<rest>' -> {rest: array}."""
    return {k[len(prefix):]: d[k] for k in d.files if k.startswith(prefix)}


def rel_err(y, ref):
    y = np.asarray(y, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return float(np.abs(y - ref).max() / max(np.abs(ref).max(), 1e-30))


def model_tol(ref32_err):
    """Whole-model parity bar of SURVEY §8(c): max|y - y64| / max|y64| <=
    max(1e-4, 2 x the reference's own fp32-vs-fp64 error on the same input)."""
    return max(1e-4, 2.0 * float(ref32_err))


@pytest.fixture(scope="session")
def golden():
    return load_npz


def _ensure_native_built():
    """Build libdstd_gcn.so in-tree if it is missing (hipcc cross-compiles)."""
    lib = os.path.join(PKG, "libdstd_gcn.so")
    if not os.path.exists(lib):
        import subprocess
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)


_ensure_native_built()
