import os
import sys

import pytest

# torch ships its own HIP runtime under the same soname (libamdhip64.so.7) as the /opt/rocm one
# libnwcrypto.so links.  Whichever library is loaded FIRST provides the runtime for both; with
# libnwcrypto's loaded first torch reports "No HIP GPUs are available" (measured on the MI355X box,
# tools/probe_runtime.sh), so torch is imported before anything loads the library.
try:
    import torch  # noqa: F401
except ImportError:   # pragma: no cover - torch is part of the image
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libnwcrypto.so")


@pytest.fixture(scope="session", autouse=True)
def _torch_gpu_first(request):
    """GPU sessions: let torch (which bundles its own HIP runtime) initialise the device before
    libnwcrypto's runtime does; in the other order torch reports "No HIP GPUs are available".
    bench.py does the same (torch.cuda.set_device before the first Engine)."""
    if any(item.get_closest_marker("gpu") is not None for item in request.session.items):
        import torch
        torch.cuda.set_device(0)
        torch.zeros(1, device="cuda:0")
    yield


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def engine():
    from narwhal_amd import _lib
    return _lib.default_engine()
