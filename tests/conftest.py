import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "omnireduce-rdma-demo_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def _ensure_built():
    """Build the oracle (gcc) and libomr.so (hipcc, gfx950) in-tree if a fresh checkout lacks them."""
    import shutil
    import subprocess
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s"], check=True)
    have_hipcc = shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")
    if have_hipcc and not os.path.exists(os.path.join(PKG, "omr", "libomr.so")):
        subprocess.run(["make", "-C", PKG, "-s"], check=True)
    if have_hipcc and not os.path.exists(os.path.join(PKG, "bin", "omr_client")):
        subprocess.run(["make", "-C", PKG, "-s", "host"], check=True)  # ./omr_client, ./omr_server
    if have_hipcc and not os.path.exists(os.path.join(ROOT, "tests", "integration", "worker_partition")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "integration"), "-s"], check=True)


def pytest_configure(config):
    _ensure_built()
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: full-size configs (seconds to minutes)")


def _has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """The HIP device; a gpu-marked test that runs without one fails loudly rather than skipping."""
    import torch
    if not _has_gpu():
        pytest.fail("gpu test started without a visible HIP device")
    import omr
    omr.load()
    return torch.device("cuda:0")
