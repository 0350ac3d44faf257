import os
import sys

# before anything initialises the HIP runtime (torch.cuda.is_available() in the hooks below):
# HIP-graph replays need the CLR's ordinary graph-launch path (visual_onoma_to_wave_amd/train.py)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def pytest_runtest_setup(item):
    if item.get_closest_marker("gpu") is not None:
        import torch
        if not torch.cuda.is_available():
            pytest.skip("needs a GPU")
