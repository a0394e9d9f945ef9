"""Build the gfx950 HIP library (``libcram_attn.so``) in-tree.

The library is the C-ABI declared in ``include/cram_attn.h``; it is compiled
directly with ``hipcc --offload-arch=gfx950`` (no torch extension machinery, no
JIT cache) so the built ``.so`` travels with the repository snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
LIB_PATH = PKG_DIR / "libcram_attn.so"
SOURCES = [CSRC / "cram_attn.hip", CSRC / "cram_fused.hip", CSRC / "cram_gemm.hip", CSRC / "cram_spans.cpp"]
HEADERS = [REPO_DIR / "include" / "cram_attn.h", CSRC / "prefill_x64.inc"]
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the CrAM HIP library cannot be built")


def needs_build() -> bool:
    if not LIB_PATH.exists():
        return True
    mtime = LIB_PATH.stat().st_mtime
    return any(p.stat().st_mtime > mtime for p in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile ``libcram_attn.so`` for gfx950 if it is missing or stale."""
    if not force and not needs_build():
        return LIB_PATH
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = [
        _hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
        "-Wall", "-Wno-unused-function",
        "-I", str(REPO_DIR / "include"),
        *[str(s) for s in SOURCES], "-o", str(tmp),
    ]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
