import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP device)')
    config.addinivalue_line('markers', 'slow: long-running test')
    # build the in-tree extension once per session (cached; no-op when up to date)
    from upow_amd import _build
    _build.build(verbose=False)


@pytest.fixture(scope='session')
def native():
    from upow_amd.ops.native import lib
    return lib()


@pytest.fixture(scope='session')
def gpu(native):
    from upow_amd.ops.native import gpu_available
    if not gpu_available():
        pytest.fail('gpu-marked test ran without a visible HIP device')
    import torch
    torch.cuda.set_device(0)
    return native
