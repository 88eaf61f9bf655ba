import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import gfa_import  # noqa: E402,F401  (registers the package as ``gfa_amd``)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libmiattack.so")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU (run with -m 'not gpu')")
    from gfa_amd import _lib
    _lib.load()  # fail loudly if the library is missing: no fallback path exists
    return torch.device("cuda:0")


def pytest_make_parametrize_id(config, val, argname):
    # readable ids for torch dtypes (-k float32 / float16 / bfloat16 select a precision)
    try:
        import torch
        if isinstance(val, torch.dtype):
            return str(val).replace("torch.", "")
    except Exception:
        pass
    return None


@pytest.fixture
def tune(cuda):
    """Set libmiattack kernel-variant switches for one test (mia_set_tuning), restored after."""
    from gfa_amd import _lib
    saved = {}

    def set_(name, value):
        old = _lib.set_tuning(name, int(value))
        saved.setdefault(name, old)
    yield set_
    for name, old in saved.items():
        _lib.set_tuning(name, old)
