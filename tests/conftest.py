import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_PARENT = os.path.join(ROOT, "hilbert-quantization_amd")
for p in (ROOT, PKG_PARENT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = load_golden(name)
        return cache[name]

    return get


@pytest.fixture(scope="session")
def hq_lib():
    """The HIP C-ABI library on a GPU box; GPU tests fail loudly if it is missing."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU in this container")
    from hq_mi355x import _lib
    return _lib.lib()


@pytest.fixture
def hq_option():
    """set(name, value) selects a kernel variant (hq_set_option) for this test; every option it touched
    is restored to its default afterwards."""
    from hq_mi355x import _lib
    touched = []

    def set_(name, value=None):
        touched.append(name)
        if value is None:
            _lib.reset_option(name)
        else:
            _lib.set_option(name, int(value))

    yield set_
    for name in touched:
        _lib.reset_option(name)
