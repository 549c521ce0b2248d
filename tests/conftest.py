import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "mjlab-1_amd"), os.path.join(ROOT, "tests"), ROOT):
  if p not in sys.path:
    sys.path.insert(0, p)


def pytest_configure(config):
  config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libmjx355.so")
  config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def gpu_device():
  import torch
  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  return "cuda:0"
