import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); runs on the GPU box")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def pytest_sessionfinish(session, exitstatus):
    from tests import _parity_report
    _parity_report.dump()


_OPTIONS = (0, 3, 5, 11, 19, 20, 24, 25, 27, 28, 29, 30, 31, 32, 33, 34)  # enum mpgnn_option switches a test may override
_DEFAULTS: dict = {}


@pytest.fixture(autouse=True)
def _restore_library_options():
    """Every test starts from the SHIPPED option values (read once, before any test changed
    them) and a test that overrides one cannot leak it into the rest of the session."""
    from mpgnn_amd import _lib
    if not _DEFAULTS:
        # MPGNN_GEMM_BF3=0|1: the whole session on the fp32-MFMA or the bf16-split GEMMs (A/B)
        v = os.environ.get("MPGNN_GEMM_BF3")
        if v is not None:
            _lib.set_option(24, int(v))
        for o in _OPTIONS:
            try:
                _DEFAULTS[o] = _lib.get_option(o)
            except (NotImplementedError, RuntimeError):  # host-only sanitizer library: no kernel options
                pass
    yield
    for o, v in _DEFAULTS.items():
        _lib.set_option(o, v)
    # kernel switches are per plan: drop the layer classes' cached plans, which may carry a
    # switch the test set on them
    from mpgnn_amd import plan_cache
    plan_cache.clear()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name))
    return load
