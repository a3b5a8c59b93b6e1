import os
import sys

import pytest

# the suite runs synthetic (random-init) models of the real architectures and
# has no network: tests of the provisioning contract unset these themselves
os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
os.environ.setdefault("SDAAS_OFFLINE", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libcsk.so")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from chiaswarm_amd.ops import _lib

    _lib.load()  # the HIP path must load on a GPU box: fail loudly otherwise
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _csk_debug_records(request):
    """With CSK_DEBUG=1 (libcsk_debug.so), every GPU test must leave no
    device-side bounds record (csrc/kernels/common.h CSK_DCHECK)."""
    yield
    if "gpu" not in request.keywords:
        return
    from chiaswarm_amd.ops import _lib

    if not _lib.DEBUG or _lib._LIB is None:
        return
    import torch

    torch.cuda.synchronize()
    recs = _lib.debug_records()
    assert not recs, f"CSK_DEBUG bounds violations (tu, count, site, block, thread, value, limit, block_y): {recs}"
