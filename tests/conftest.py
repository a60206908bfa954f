import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmk.so on cuda:0)")


@pytest.fixture(scope="session")
def mk():
    return importlib.import_module(PKG)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
