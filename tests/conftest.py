import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import mpisppy_amd  # noqa: E402,F401  (registers the package alias)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the real libphx kernels)")


EMU_PATH = os.path.join(ROOT, "tests", "emu", "libphx_emu.so")


@pytest.fixture(scope="session")
def emu():
    """Test-only host emulation of the phx ABI (same per-lane math as the kernels)."""
    from mpisppy_amd import _native
    from mpisppy_amd import build as b
    b.build_emu(verbose=False)
    return _native.Lib(EMU_PATH, prefix="emu_phx_")


@pytest.fixture(scope="session")
def gpu_lib():
    import torch
    from mpisppy_amd import _native
    if not torch.cuda.is_available():
        pytest.fail("gpu test on a machine without a GPU")
    return _native.load()
