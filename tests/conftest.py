import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no GPU is visible")
    from cram_amd import build
    build.build()
    return torch.device("cuda:0")


@pytest.fixture(params=["bk64", "bk32", "w8"])
def prefill_variant(request, monkeypatch):
    """Run a prefill test on every d=128 prefill kernel: the default 64-key tiles at two waves per SIMD, the
    opt-in 32-key tiles at three (CRAM_PREFILL_VARIANT=3) and the 8-wave workgroups (=8).  The library reads
    the variable at every launch."""
    if request.param in ("bk32", "w8"):
        monkeypatch.setenv("CRAM_PREFILL_VARIANT", {"bk32": "3", "w8": "8"}[request.param])
    else:
        monkeypatch.delenv("CRAM_PREFILL_VARIANT", raising=False)
    return request.param


@pytest.fixture(params=["auto", "u1", "u2"])
def decode_variant(request, monkeypatch):
    """Run a decode test on every decode_kernel instantiation: the size-picked keys-per-iteration U (1 for grids of
    >= 1024 workgroups, else 4) and the forced U = 1 / 2 (CRAM_DECODE_U, read at every launch)."""
    if request.param == "auto":
        monkeypatch.delenv("CRAM_DECODE_U", raising=False)
    else:
        monkeypatch.setenv("CRAM_DECODE_U", request.param[1])
    return request.param
