import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

# HL_LIB=<path>: run the GPU tests against another build of the product
# library (debug builds such as `make poison`); the default is the in-tree one.
if os.environ.get("HL_LIB"):
    from hartallo_amd import _lib as _hl_lib

    _hl_lib.load_library(os.path.abspath(os.environ["HL_LIB"]))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity of the HIP path against the oracle")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not _gpu_available():
        pytest.fail("no GPU visible: the gfx950 path has no CPU fallback")
    return True
