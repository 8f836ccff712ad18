import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _ensure_built():
    lib = os.path.join(ROOT, "deneva_amd", "libdcc.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(ROOT, "deneva_amd", "csrc"), "-j8"], check=True)


_ensure_built()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def engine():
    if not gpu_available():
        pytest.skip("no GPU")
    from deneva_amd import Engine
    e = Engine(0)
    yield e
    e.close()
