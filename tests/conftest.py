import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "sketches-py_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def built_lib():
    """Path of libgkarray_hip.so, building it in-tree if it is missing."""
    import subprocess
    so = os.path.join(ROOT, "sketches-py_amd", "gkarray_amd", "libgkarray_hip.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-j8", "-C", os.path.join(ROOT, "sketches-py_amd", "csrc")],
                       check=True, stdout=subprocess.DEVNULL)
    return so


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
