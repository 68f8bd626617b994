import os
import pathlib
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO / "genome-assembly_amd"))
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- run with -m gpu")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def digests():
    import json
    return json.loads((GOLDEN / "digests.json").read_text())


@pytest.fixture(params=["table", "binned"])
def engine(request, monkeypatch):
    """KB_ENGINE for the case: the binned engine applies to K <= 63 (two-word
    k-mers on its bucketed path: reads <= 512 bp); elsewhere the table engine
    runs either way"""
    monkeypatch.setenv("KB_ENGINE", request.param)
    return request.param
