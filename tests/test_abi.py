"""The C-ABI library loads (no GPU needed) and exports exactly what include/cram_attn.h declares."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(REPO, "include", "cram_attn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cram_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = _declared()
    for n in ("cram_attn_prefill", "cram_attn_decode", "cram_attn_decode_shared", "cram_attn_decode_workspace_size", "cram_answer_logits",
              "cram_strerror", "cram_abi_version", "cram_rmsnorm", "cram_rope_inplace", "cram_rope_split", "cram_silu_mul",
              "cram_gemm", "cram_gemm_residual", "cram_gemm_rope"):
        assert n in names


def test_library_builds_loads_and_exports_every_symbol():
    from cram_amd import build, _lib
    build.build()
    lib = ctypes.CDLL(str(build.LIB_PATH))
    for n in _declared():
        assert hasattr(lib, n), n
    assert set(_declared()) == set(_lib.SIGNATURES), "ctypes signatures must cover the header exactly"
    L = _lib.load()
    assert L.cram_abi_version() == _lib.ABI_VERSION == 8
    assert L.cram_strerror(-3) == b"stride not a multiple of 8 elements or pointer not 16-byte aligned"
    assert L.cram_attn_decode_workspace_size(2, 32, 128, 4) == 2 * 32 * 4 * 130 * 4
    assert L.cram_attn_decode_workspace_size(2, 32, 128, 1) == 0


def test_argument_validation_without_gpu():
    """Bad arguments are rejected on the host before any launch (no device needed)."""
    from cram_amd import _lib
    L = _lib.load()
    # null pointers
    assert L.cram_attn_prefill(None, 0, 0, 0, None, 0, 0, 0, None, 0, 0, 0, None, 0, 0, 0,
                               1, 1, 1, 1, 1, 128, 0, 1.0, None, 0, None, 0, 0, 0, None) == -1
    # unsupported head dim (checked before alignment / launch)
    fake = 1 << 20
    assert L.cram_attn_prefill(fake, 0, 0, 0, fake, 0, 0, 0, fake, 0, 0, 0, fake, 0, 0, 0,
                               1, 1, 1, 1, 1, 96, 0, 1.0, None, 0, None, 0, 0, 0, None) == -2
    # unsupported element type (only CRAM_DTYPE_BF16 = 0 and CRAM_DTYPE_F16 = 1)
    assert L.cram_attn_prefill(fake, 0, 0, 0, fake, 0, 0, 0, fake, 0, 0, 0, fake, 0, 0, 0,
                               1, 1, 1, 1, 1, 128, 0, 1.0, None, 0, None, 0, 0, 2, None) == -2
    assert L.cram_silu_mul(fake, 8, fake, 8, 1, 16, 7, None) == -2
    # misaligned stride
    assert L.cram_attn_prefill(fake, 8, 8, 12, fake, 0, 0, 8, fake, 0, 0, 8, fake, 0, 0, 8,
                               1, 1, 1, 1, 1, 128, 0, 1.0, None, 0, None, 0, 0, 1, None) == -3
    # split decode without workspace
    assert L.cram_attn_decode(fake, 0, 0, fake, 0, 0, 8, fake, 0, 0, 8, fake, 0, 0,
                              1, 1, 1, 4, None, 128, 1.0, None, 0, None, 0, 0, 4, None, 0, 0, None) == -5
    assert L.cram_rmsnorm(None, 0, None, 0, None, 0, None, None, 0, 1, 8, 1e-5, 0, None) == -1
    assert L.cram_silu_mul(fake, 8, fake, 8, 1, 12, 0, None) == -3
    # projection GEMM: N % 256, K % 64, row alignment, epilogue code, output row length
    assert L.cram_gemm(fake, 64, fake, 64, fake, 256, 1, 200, 64, 0, 0, None) == -2
    assert L.cram_gemm(fake, 48, fake, 48, fake, 256, 1, 256, 48, 0, 0, None) == -2
    assert L.cram_gemm(fake, 68, fake, 64, fake, 256, 1, 256, 64, 0, 0, None) == -3
    assert L.cram_gemm(fake, 64, fake, 64, fake, 256, 1, 256, 64, 2, 0, None) == -1
    assert L.cram_gemm(fake, 64, fake, 64, fake, 128, 1, 512, 64, 0, 0, None) == -1
    # residual GEMM: residual presence and alignment, overlap other than exact aliasing, then cram_gemm's checks
    far = 1 << 24
    assert L.cram_gemm_residual(fake, 64, fake, 64, None, 256, fake, 256, 1, 256, 64, 0, None) == -1
    assert L.cram_gemm_residual(fake, 64, fake, 64, far, 260, fake, 256, 1, 256, 64, 0, None) == -3
    assert L.cram_gemm_residual(fake, 64, fake, 64, far + 8, 256, fake, 256, 1, 256, 64, 0, None) == -3
    assert L.cram_gemm_residual(fake, 64, fake, 64, fake + 16, 256, fake, 256, 1, 256, 64, 0, None) == -1
    assert L.cram_gemm_residual(fake, 64, fake, 64, far, 256, fake, 256, 0, 256, 64, 0, None) == -1
    assert L.cram_gemm_residual(fake, 64, fake, 64, far, 256, fake, 256, 1, 200, 64, 0, None) == -2
    assert L.cram_gemm_residual(fake, 64, fake, 64, fake, 256, fake, 256, 1, 256, 48, 0, None) == -2
    # q/k/v + RoPE GEMM: tables, rows <= M, kout / vout together, dst_b needs pos, bf16 and head dim 128 only
    def rope(M=256, K=128, rows=256, T=256, d=128, cos=fake, kout=None, vout=None, dst_b=None, pos=None, dtype=0,
             ldo=6144):
        return L.cram_gemm_rope(fake, K, fake, K, None, fake, ldo, M, K, rows, T, 32, 8, d, cos, fake, 128, pos, 0,
                                kout, vout, 0, 0, 0, 0, dst_b, 0, dtype, None)
    assert rope(cos=None) == -1
    assert rope(rows=257) == -1
    assert rope(kout=fake) == -1
    assert rope(kout=fake, vout=fake, dst_b=fake) == -1
    assert rope(kout=fake, vout=fake, rows=200, T=64) == -1
    assert rope(d=64) == -2
    assert rope(dtype=2) == -2
    assert rope(K=64) == -2
    assert rope(ldo=6148) == -3
    assert L.cram_gemm_rope(fake, 128, fake, 128, fake + 8, fake, 6144, 256, 128, 256, 256, 32, 8, 128, fake, fake, 128,
                            None, 0, None, None, 0, 0, 0, 0, None, 0, 0, None) == -3      # misaligned bias
    # split-K residual: residual checks, then split-K's (workspace)
    ws4 = L.cram_gemm_splitk_workspace_size(16, 512, 4)
    assert L.cram_gemm_splitk_residual(fake, 512, fake, 512, None, 512, fake, 512, 16, 512, 512, 4, fake, ws4, 0,
                                       None) == -1
    assert L.cram_gemm_splitk_residual(fake, 512, fake, 512, far, 516, fake, 512, 16, 512, 512, 4, fake, ws4, 0,
                                       None) == -3
    assert L.cram_gemm_splitk_residual(fake, 512, fake, 512, fake + 1024, 512, fake, 512, 16, 512, 512, 4, fake, ws4,
                                       0, None) == -1
    assert L.cram_gemm_splitk_residual(fake, 512, fake, 512, far, 512, fake, 512, 16, 512, 512, 4, None, ws4, 0,
                                       None) == -5
    # split-K GEMM: K % (64 * splits), epilogue, bias only with STORE, workspace presence and size
    ws = L.cram_gemm_splitk_workspace_size(16, 512, 4)
    assert ws == 4 * 16 * 512 * 4
    assert L.cram_gemm_splitk(fake, 512, fake, 512, fake, 512, 16, 512, 512, 3, 0, None, fake, ws, 0, None) == -2
    assert L.cram_gemm_splitk(fake, 512, fake, 512, fake, 512, 16, 512, 512, 4, 1, None, fake, ws, 0, None) == -1
    assert L.cram_gemm_splitk(fake, 512, fake, 512, fake, 512, 16, 512, 512, 4, 2, fake, fake, ws, 0, None) == -1
    assert L.cram_gemm_splitk(fake, 512, fake, 512, fake, 512, 16, 512, 512, 4, 0, None, None, ws, 0, None) == -5
    assert L.cram_gemm_splitk(fake, 512, fake, 512, fake, 512, 16, 512, 512, 4, 0, None, fake, ws - 1, 0, None) == -5
    assert L.cram_gemm_splitk(fake, 512, fake, 512, fake, 260, 16, 512, 512, 4, 2, None, fake, ws, 0, None) == -3


def test_kernel_knobs_latch_without_gpu():
    """Kernel selection is a process-wide knob (read from the environment once, never per launch)."""
    from cram_amd import _lib
    L = _lib.load()
    prev = _lib.set_knob(_lib.KNOB_DECODE_U, 2)
    try:
        assert _lib.get_knob(_lib.KNOB_DECODE_U) == 2
        os.environ["CRAM_DECODE_U"] = "4"            # the environment is not re-read after the first query
        assert _lib.get_knob(_lib.KNOB_DECODE_U) == 2
        with pytest.raises(RuntimeError):
            _lib.set_knob(_lib.KNOB_PREFILL_VARIANT, 5)
        # an unknown knob is an error code distinct from every knob value (-1 = automatic is a value)
        v = ctypes.c_int(123)
        assert L.cram_get_knob(99, ctypes.byref(v)) == -1 and v.value == 123
        assert L.cram_get_knob(_lib.KNOB_DECODE_U, None) == -1
        assert _lib.set_knob(_lib.KNOB_DECODE_MFMA, -1) in (-1, 0, 1) and _lib.get_knob(_lib.KNOB_DECODE_MFMA) == -1
    finally:
        os.environ.pop("CRAM_DECODE_U", None)
        _lib.set_knob(_lib.KNOB_DECODE_U, prev)


def test_product_path_fails_loudly_without_library(tmp_path, monkeypatch):
    from cram_amd import _lib
    monkeypatch.setattr(_lib, "_LIB", None)
    monkeypatch.setattr(_lib, "LIB_PATH", tmp_path / "missing.so")
    with pytest.raises(_lib.CrAMLibraryError):
        _lib.load()


def test_plain_c_host_builds_and_links():
    """examples/abi_demo.c: the header compiles as C11 and links against libcram_attn.so + the HIP runtime."""
    import shutil
    import subprocess
    from cram_amd import build
    build.build()
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    ex = os.path.join(REPO, "examples")
    subprocess.run(["make", "-C", ex, "-s", "clean"], check=True)
    subprocess.run(["make", "-C", ex, "-s"], check=True)
    assert os.access(os.path.join(ex, "abi_demo"), os.X_OK)
