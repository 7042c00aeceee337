import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); run with -m gpu")
    config.addinivalue_line("markers", "slow: multi-process / long-running CPU test")


def pytest_collection_modifyitems(config, items):
    # child-process-only GPU tests first, while the pytest process has not brought HIP up yet (the
    # in-process tests' session fixture creates a context that then lives to the end)
    items.sort(key=lambda it: 0 if "gpu_box" in getattr(it, "fixturenames", ()) else 1)


@pytest.fixture(scope="session")
def gpu_box():
    """A GPU is usable, checked WITHOUT bringing HIP up in the pytest process: for tests whose GPU work
    runs in child processes only (several ranks on one GPU - an idle context in the parent would hold
    hardware queues of its own beside the ranks' spinning all-reduce kernels)."""
    from pytorch_mnist_ddp_amd.driver import gpu_present
    if not gpu_present():
        pytest.skip("no GPU")
    return True


@pytest.fixture(scope="session")
def cuda_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def init_world1_pg(backend, device=None):
    """world_size=1 process group over a TCPStore bound to an OS-chosen port (port 0): no
    pick-a-free-port-then-bind race with other jobs on the box (EADDRINUSE)."""
    import datetime

    import torch.distributed as dist
    store = dist.TCPStore("127.0.0.1", 0, 1, True, timeout=datetime.timedelta(seconds=60))
    kw = {"device_id": device} if device is not None else {}
    dist.init_process_group(backend, store=store, world_size=1, rank=0, **kw)
    return store
