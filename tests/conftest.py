import os
import sys

# Stage and copy streams of a multi-partition Pipe on one GPU must not alias
# onto shared in-order hardware queues (HIP's default is 4; see
# profiles/hw_queue_sharing.txt): read by HIP at initialisation, so set it
# before anything touches the GPU.  The GPU boxes export HIP's default (4)
# explicitly; any other explicit setting wins.
if os.environ.get("GPU_MAX_HW_QUEUES", "4") in ("", "4"):
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) device")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs in one process")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(autouse=True)
def manual_seed_zero():
    torch.manual_seed(0)


@pytest.fixture
def cuda_sleep():
    """Returns sleep(seconds) that enqueues a busy-wait kernel on the current
    stream -- used to prove that streams overlap (upstream conftest idea)."""
    from mipipe import _native_loader

    k = _native_loader.kernels()

    def sleep(seconds: float) -> None:
        k.gpu_sleep(int(seconds * 1e6))

    return sleep


def pytest_collection_modifyitems(config, items):
    have_gpu = torch.cuda.is_available()
    ngpu = torch.cuda.device_count() if have_gpu else 0
    skip_gpu = pytest.mark.skip(reason="no GPU")
    skip_multi = pytest.mark.skip(reason="needs >= 2 GPUs")
    for item in items:
        if "gpu" in item.keywords and not have_gpu:
            item.add_marker(skip_gpu)
        if "multigpu" in item.keywords and ngpu < 2:
            item.add_marker(skip_multi)
