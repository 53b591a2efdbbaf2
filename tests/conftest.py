import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.dont_write_bytecode = True


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (ROCm GPU) and libddmi.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda.is_available() is False")
    from diffusiondrive_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def seeded_sd():
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.weights import seeded_state_dict
    return seeded_state_dict(TransfuserConfig(), 0)


@pytest.fixture(scope="session")
def gpu_model(gpu, seeded_sd):
    from diffusiondrive_amd.model import DiffusionDriveModel
    return DiffusionDriveModel(state_dict=seeded_sd, device=0)
