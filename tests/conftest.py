import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built native extension")
    config.addinivalue_line("markers", "slow: multi-process / long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pytorch_distributed_examples_amd import _native

    _native.C()  # fail loudly if the extension is missing on a GPU box
    return torch.device("cuda:0")
