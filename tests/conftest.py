import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
# the specialised kernels' on-disk code-object cache stays inside the tree
os.environ.setdefault("WOLOLO_JIT_CACHE", os.path.join(ROOT, ".jit_cache"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _have_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _have_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session", autouse=True)
def built_libraries():
    """Build libwololo.so and the oracle once per session (no-op when up to date)."""
    lib = os.path.join(ROOT, "csgrenderer_amd", "lib", "libwololo.so")
    if not os.path.exists(lib) or os.environ.get("WOLOLO_REBUILD"):
        subprocess.run(["make", "-C", os.path.join(ROOT, "csgrenderer_amd", "csrc"), "-j8"], check=True,
                       stdout=subprocess.DEVNULL)
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    yield


@pytest.fixture()
def hostonly(monkeypatch):
    """Device-less renderer (node store + compiler only) for CPU tests."""
    monkeypatch.setenv("WOLOLO_ALLOW_NO_DEVICE", "1")
    yield
