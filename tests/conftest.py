import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:       # test-only helper modules (e.g. map_reference_impl)
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    # host torch ops of the (small) test problems: intra-op threads beyond a few cost more than they give on
    # shared vCPUs (softplus of a 4500 x 32 block: 1.9 ms on 1 thread, 13.5 ms on 8 here), and xdist workers
    # each spin their own pool; TMOG_TEST_THREADS overrides
    try:
        import torch
        torch.set_num_threads(int(os.environ.get("TMOG_TEST_THREADS", "1")))
    except Exception:
        pass
    config.addinivalue_line("markers", "gpu: test needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _reset_uid():
    from transmogrifai_amd import uid
    uid.reset(0)
    yield
