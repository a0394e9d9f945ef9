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


@pytest.fixture(params=["bk64", "bk32", "w8", "hp7", "x32"])
def prefill_variant(request):
    """Run a prefill test on every d=128 prefill kernel: the 4-wave 64-key tiles at two waves per SIMD (variant 0), the
    opt-in 32-key tiles at three (variant 3), the 8-wave workgroups (variant 8), the 7-wave GQA-7 workgroups
    (variant 7; the automatic choice for GQA-7 up to 2048 tokens) and the hand-scheduled two-workgroups-per-CU kernel
    with 32 rows per wave (variant 4: bf16 GQA groups of 4k, the automatic choice from 256 rows; other shapes fall
    back to variant 0), selected through the library's process-wide knob (cram_set_knob)."""
    from cram_amd import _lib
    prev = _lib.set_knob(_lib.KNOB_PREFILL_VARIANT, {"bk64": 0, "bk32": 3, "w8": 8, "hp7": 7, "x32": 4}[request.param])
    yield request.param
    _lib.set_knob(_lib.KNOB_PREFILL_VARIANT, prev)


@pytest.fixture(params=["auto", "valu_u1", "valu_u2", "valu_u4"])
def decode_variant(request):
    """Run a decode test on every decode body: the automatic choice (matrix-core kernel for GQA groups of >= 4 heads
    at d = 128, else the VALU kernel with its size-picked U) and the VALU kernel forced with U = 1 / 2 / 4 keys per
    lane group (knobs CRAM_KNOB_DECODE_MFMA = 0, CRAM_KNOB_DECODE_U)."""
    from cram_amd import _lib
    mf, u = (-1, -1) if request.param == "auto" else (0, int(request.param[-1]))
    prev = (_lib.set_knob(_lib.KNOB_DECODE_MFMA, mf), _lib.set_knob(_lib.KNOB_DECODE_U, u))
    yield request.param
    _lib.set_knob(_lib.KNOB_DECODE_MFMA, prev[0])
    _lib.set_knob(_lib.KNOB_DECODE_U, prev[1])
