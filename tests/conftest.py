import os
import sys

import pytest

# the GPU tests run with the hardware-queue count bench.py uses (streams on separate queues really
# run concurrently: this is what exposed the missing side-stream wait of synchronous bucketed
# clocks); set before anything imports torch
if os.environ.get("GPU_MAX_HW_QUEUES", "4") == "4":  # unset or HIP's default (the GPU box exports 4)
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MINIPS_HW_QUEUES", "8")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
