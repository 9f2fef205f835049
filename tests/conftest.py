import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def pytest_collection_modifyitems(config, items):
    """A test that takes the `gpu` fixture without the `gpu` marker would be
    skipped on CPU and deselected by `-m gpu`, i.e. never run: refuse it."""
    unmarked = [it.nodeid for it in items
                if "gpu" in getattr(it, "fixturenames", ()) and it.get_closest_marker("gpu") is None]
    if unmarked:
        raise pytest.UsageError("tests use the gpu fixture without @pytest.mark.gpu: " + ", ".join(unmarked))


@pytest.fixture
def table_kernels():
    """Pointer-table calls take the table kernels even when their shards form a
    slot grid (knob ptrs_grid=0): for tests of the table path itself (table
    cache, upload chunks, the table kernels of the sweep)."""
    import shmr_amd
    shmr_amd.set_tuning(ptrs_grid=0)
    try:
        yield
    finally:
        shmr_amd.set_tuning(ptrs_grid=-2)
