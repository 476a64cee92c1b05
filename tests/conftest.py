import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs on the GPU box)')
    config.addinivalue_line('markers', 'slow: longer CPU test')


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason='no GPU in this container')
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def mb_off():
    """The split form's 16x16x4 instances for the whole test (fs_tuning.split_mb = -1): the modules
    that hold the pair, pipe, team and double-buffered forms BITWISE to the split form compare
    within that family -- the mb instances (4x4x1 MFMAs, another summation order) are held to the
    oracle in test_gpu_mb.py."""
    from fedamw_amd import _lib
    with _lib.tuning(split_mb=-1):
        yield
