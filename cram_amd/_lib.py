"""ctypes binding of ``libcram_attn.so`` (the C-ABI of ``include/cram_attn.h``).

There is no fallback: if the HIP library is missing the product path raises.
torch is imported first so that the HIP runtime torch ships
(``libamdhip64.so.7``) is the one the library binds to.
"""
from __future__ import annotations

import ctypes
from ctypes import c_float, c_int, c_int64, c_size_t, c_void_p, POINTER

import torch  # noqa: F401  (loads the HIP runtime before the library)

from .build import LIB_PATH

_c_int32_p = POINTER(ctypes.c_int32)
_c_uint8_p = POINTER(ctypes.c_uint8)
_c_float_p = POINTER(c_float)

ABI_VERSION = 8   # CRAM_ABI_VERSION of include/cram_attn.h

# name -> (restype, argtypes); the exact export list of include/cram_attn.h
SIGNATURES = {
    "cram_strerror": (ctypes.c_char_p, [c_int]),
    "cram_abi_version": (c_int, []),
    "cram_set_knob": (c_int, [c_int, c_int]),
    "cram_get_knob": (c_int, [c_int, c_void_p]),
    "cram_attn_prefill": (c_int, [
        c_void_p, c_int64, c_int64, c_int64,
        c_void_p, c_int64, c_int64, c_int64,
        c_void_p, c_int64, c_int64, c_int64,
        c_void_p, c_int64, c_int64, c_int64,
        c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
        c_void_p, c_int64, c_void_p, c_int64, c_int,
        c_int, c_void_p,
    ]),
    "cram_attn_prefill_varlen": (c_int, [
        c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64,
        c_void_p, c_int64, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int, c_float,
        c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_void_p,
    ]),
    "cram_attn_prefill_varlen_cached": (c_int, [
        c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64, c_int64, c_int64,
        c_void_p, c_int64, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
        c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_void_p,
    ]),
    "cram_attn_decode_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int]),
    "cram_attn_decode": (c_int, [
        c_void_p, c_int64, c_int64,
        c_void_p, c_int64, c_int64, c_int64,
        c_void_p, c_int64, c_int64, c_int64,
        c_void_p, c_int64, c_int64,
        c_int, c_int, c_int, c_int, c_void_p, c_int, c_float,
        c_void_p, c_int64, c_void_p, c_int64, c_int,
        c_int, c_void_p, c_size_t,
        c_int, c_void_p,
    ]),
    "cram_attn_decode_shared": (c_int, [
        c_void_p, c_int64, c_int64,
        c_void_p, c_int64, c_int64, c_int64,
        c_void_p, c_int64, c_int64, c_int64,
        c_void_p, c_int64, c_int64,
        c_int, c_int, c_int, c_int, c_void_p, c_int, c_float,
        c_void_p, c_int64, c_void_p, c_int64, c_int,
        c_int, c_int, c_void_p, c_size_t,
        c_int, c_void_p,
    ]),
    "cram_answer_logits": (c_int, [
        c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
    ]),
    "cram_rmsnorm": (c_int, [
        c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_int,
        c_float, c_int, c_void_p,
    ]),
    "cram_rope_inplace": (c_int, [
        c_void_p, c_int64, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_void_p,
    ]),
    "cram_rope_split": (c_int, [
        c_void_p, c_int64, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
        c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p, c_int, c_int, c_void_p,
    ]),
    "cram_silu_mul": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_int, c_void_p]),
    "cram_gemm": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_int, c_int, c_int,
                          c_void_p]),
    "cram_gemm_residual": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int,
                                   c_int, c_int, c_int, c_void_p]),
    "cram_gemm_rope": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_int, c_int,
                               c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_void_p,
                               c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p, c_int, c_int, c_void_p]),
    "cram_gemm_small": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_int, c_int,
                                c_int, c_int, c_void_p, c_size_t, c_int, c_void_p]),
    "cram_gemm_splitk_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cram_gemm_splitk": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_int, c_int,
                                 c_int, c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    "cram_gemm_splitk_residual": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                          c_int, c_int, c_int, c_int, c_void_p, c_size_t, c_int, c_void_p]),
    "cram_passage_weights": (c_int, [c_int] + [c_void_p] * 9),
}

_LIB = None


class CrAMLibraryError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load the HIP library (raises if it has not been built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not LIB_PATH.exists():
        raise CrAMLibraryError(
            f"{LIB_PATH} is missing: build it with `python -m cram_amd.build` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.cram_abi_version() != ABI_VERSION:
        raise CrAMLibraryError(f"{LIB_PATH} exports ABI {lib.cram_abi_version()}, this binding needs {ABI_VERSION}: "
                               "rebuild it with `python -m cram_amd.build`")
    _LIB = lib
    return lib


def check(code: int, what: str) -> None:
    if code != 0:
        msg = load().cram_strerror(code).decode()
        raise RuntimeError(f"{what} failed: CRAM error {code} ({msg})")


KNOB_PREFILL_VARIANT = 0   # CRAM_KNOB_PREFILL_VARIANT
KNOB_DECODE_U = 1          # CRAM_KNOB_DECODE_U
KNOB_DECODE_MFMA = 2       # CRAM_KNOB_DECODE_MFMA
KNOB_GEMM_VARIANT = 3      # CRAM_KNOB_GEMM_VARIANT


def set_knob(which: int, value: int) -> int:
    """Set a process-wide kernel-selection knob (-1 = automatic); returns the previous value."""
    prev = get_knob(which)
    check(load().cram_set_knob(which, int(value)), "cram_set_knob")
    return prev


def get_knob(which: int) -> int:
    v = ctypes.c_int(0)
    check(load().cram_get_knob(which, ctypes.byref(v)), "cram_get_knob")
    return v.value
