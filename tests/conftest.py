import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (gfx950) and libogbx.so')


@pytest.fixture(scope='session')
def gpu():
    """The GPU device; GPU tests fail loudly (never skip) without one."""
    import torch

    assert torch.cuda.is_available(), 'gpu-marked test run without a visible GPU'
    from ogbench_amd import _lib

    _lib.lib()
    return torch.device('cuda', 0)


@pytest.fixture(scope='session')
def golden_locomaze():
    import numpy as np

    return dict(np.load(os.path.join(GOLDEN, 'locomaze_golden.npz')))
