"""Build the gfx950 HIP library (``libcram_attn.so``) in-tree.

The library is the C-ABI declared in ``include/cram_attn.h``; it is compiled
directly with ``hipcc --offload-arch=gfx950`` (no torch extension machinery, no
JIT cache) so the built ``.so`` travels with the repository snapshot.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
LIB_PATH = PKG_DIR / "libcram_attn.so"
SOURCES = [CSRC / "cram_attn.hip", CSRC / "cram_fused.hip", CSRC / "cram_gemm.hip", CSRC / "cram_spans.cpp"]
HEADERS = [REPO_DIR / "include" / "cram_attn.h", CSRC / "prefill_asm.inc", CSRC / "prefill_x32.inc",
           CSRC / "gemm_w4_loop.inc", CSRC / "cram_silu.inc"]
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the CrAM HIP library cannot be built")


COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]
HASH_TAG = b"CRAM_SOURCE_HASH="


def source_hash() -> str:
    """Identity of everything the library is built from: every source and header, the flags and the target."""
    import hashlib
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        h.update(f.name.encode() + b"\0" + f.read_bytes())
    h.update(" ".join(COMMON_FLAGS + [ARCH]).encode())
    return h.hexdigest()[:16]


def built_hash(path: Path = LIB_PATH):
    """The source hash a built library carries (cram_spans.cpp embeds "CRAM_SOURCE_HASH=<hash>"), or None."""
    try:
        data = path.read_bytes()
    except OSError:
        return None
    i = data.find(HASH_TAG)
    return data[i + len(HASH_TAG): i + len(HASH_TAG) + 16].decode("ascii", "replace") if i >= 0 else None


def needs_build() -> bool:
    """True unless the installed library was built from exactly the current sources (by content hash, not mtime:
    a snapshot copied with newer mtimes, or a library copied in with stale sources, is caught either way)."""
    return built_hash() != source_hash()


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile ``libcram_attn.so`` for gfx950 if it is missing or built from other sources (one hipcc process per
    source, in parallel, then one link).  Concurrent builds (two test sessions) serialise on a lock file."""
    import fcntl
    objdir = PKG_DIR / "build"
    objdir.mkdir(exist_ok=True)
    with open(objdir / ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and not needs_build():
            return LIB_PATH
        return _build(objdir, verbose)


def _build(objdir: Path, verbose: bool) -> Path:
    tmp = LIB_PATH.with_suffix(".so.tmp")
    sh = source_hash()
    common = [_hipcc(), f"--offload-arch={ARCH}", *COMMON_FLAGS, "-I", str(REPO_DIR / "include"),
              f'-DCRAM_SOURCE_HASH="{sh}"']
    objs, procs = [], []
    for src in SOURCES:
        obj = objdir / (src.name + ".o")
        # the attention library keeps its device assembly (same compile as the object) for the register audit
        extra = ["-save-temps=obj"] if src.name in ASM_SOURCES else []
        cmd = common + extra + ["-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    failed = [cmd for p, cmd in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    asm = "\n".join(asm_path(src).read_text() for src in ASM_SOURCES)
    for kname in asm_kernels(asm):
        bad = audit_asm_kernel(asm, kname)
        if bad:
            raise RuntimeError(f"{kname} register audit failed (the library is not installed): " + "; ".join(bad[:5]))
    (objdir / "asm.hash").write_text(sh)
    link = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *[str(o) for o in objs], "-o", str(tmp)]
    if verbose:
        print(" ".join(link), file=sys.stderr)
    subprocess.run(link, check=True)
    if built_hash(tmp) != sh:
        raise RuntimeError("the linked library does not carry its source hash (cram_spans.cpp tag missing)")
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


def device_asm(out_dir: Path) -> str:
    """Device assembly of the sources with register-owning kernels (ASM_SOURCES), compiled with the library's flags
    into out_dir (for the register audit without touching the installed library): the saved assembly of the last
    build when it matches the sources."""
    stamp = PKG_DIR / "build" / "asm.hash"
    if stamp.exists() and stamp.read_text().strip() == source_hash() and all(asm_path(s).exists() for s in ASM_SOURCES):
        return "\n".join(asm_path(s).read_text() for s in ASM_SOURCES)
    texts = []
    for src in ASM_SOURCES:
        out = Path(out_dir) / (src + ".s")
        subprocess.run([_hipcc(), f"--offload-arch={ARCH}", *COMMON_FLAGS, "-I", str(REPO_DIR / "include"),
                        "--cuda-device-only", "-S", str(CSRC / src), "-o", str(out)], check=True)
        texts.append(out.read_text())
    return "\n".join(texts)


def asm_path(src: str) -> Path:
    """Device assembly of a source saved by the last build (-save-temps=obj)."""
    return PKG_DIR / "build" / f"{src.rsplit('.', 1)[0]}-hip-amdgcn-amd-amdhsa-{ARCH}.s"


def kernel_source_hash() -> str:
    """Identity of the attention kernels' source (cram_attn.hip, prefill_asm.inc, prefill_x32.inc, the ABI header):
    PMC evidence (profiles/attn_pmc.json) records the hash it was measured on, and bench.py uses it only while it
    matches."""
    import hashlib
    h = hashlib.sha256()
    for f in (CSRC / "cram_attn.hip", CSRC / "prefill_asm.inc", CSRC / "prefill_x32.inc", REPO_DIR / "include" / "cram_attn.h"):
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def gemm_source_hash() -> str:
    """Identity of the projection GEMM's source (cram_gemm.hip, the generated K loop, the ABI header): the GEMM PMC
    evidence (profiles/gemm_pmc.json) records it, and bench.py applies that evidence only while it matches."""
    import hashlib
    h = hashlib.sha256()
    for f in (CSRC / "cram_gemm.hip", CSRC / "gemm_w4_loop.inc", CSRC / "cram_silu.inc",
              REPO_DIR / "include" / "cram_attn.h"):
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def x64_asm_path() -> Path:
    """Device assembly of cram_attn.hip saved by the last build (-save-temps=obj)."""
    return asm_path("cram_attn.hip")


def kernel_body(asm: str, name: str) -> str:
    m = re.search(r"^(" + name + r"):", asm, re.M) if name.startswith("_Z") else \
        re.search(r"^(_Z\w*" + name + r"\w*):", asm, re.M)
    if not m:
        raise RuntimeError(f"kernel {name} not found in the assembly")
    return asm[m.end(): asm.find(".Lfunc_end", m.end())]


def _sgprs(op: str) -> set:
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", op)
    return {int(m.group(1))} if m else set()


_NO_DST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_barrier", "s_setprio", "s_endpgm")


# kernels that own accumulator registers by name inside their inline asm: prefill_x32_kernel (O = a[0:63],
# Q = a[64:95]) and every instantiation of gemm_w4_kernel (all 256 accumulators a[0:255], its K loop one asm
# statement, the epilogue's accumulator reads separate statements -- nothing of hipcc's may touch an AGPR in between).
# The list is not written by hand: `asm_kernels` takes every symbol whose name contains one of these stems from the
# assembly, so a new epilogue or element type is audited as soon as it is instantiated.
ASM_KERNEL_STEMS = ("prefill_x32_kernel", "gemm_w4_kernel")
ASM_SOURCES = ("cram_attn.hip", "cram_gemm.hip")


def asm_kernels(asm: str) -> list:
    """Every kernel symbol of the assembly whose name contains one of ASM_KERNEL_STEMS (mangled names, sorted)."""
    stems = "|".join(ASM_KERNEL_STEMS)
    names = sorted(set(re.findall(r"^(_Z\w*(?:" + stems + r")\w*):", asm, re.M)))
    for stem in ASM_KERNEL_STEMS:
        if not any(stem in n for n in names):
            raise RuntimeError(f"no {stem} symbol in the assembly: the register audit no longer matches the sources")
    return names


def audit_asm_kernel(asm: str, kname: str = "prefill_x32_kernel") -> list:
    """The kernels of `asm_kernels` own accumulator registers by name inside their inline asm (prefill_x32_kernel:
    O = a[0:63], Q = a[64:95]; gemm_w4_kernel: a[0:255]); hipcc knows nothing of that.
    Returns the violations in kernel `kname` (empty = clean):
      * any v_accvgpr_* / AGPR operand the COMPILER emitted (outside the kernel's ;;#ASMSTART..;;#ASMEND blocks);
      * any scratch traffic in the kernel;
      * an LDS-DMA whose descriptor SGPRs were written by a VALU op fewer than 5 wait states earlier (the kernel's
        DMA pieces after the first of a tile carry no s_nop of their own)."""
    body = kernel_body(asm, kname)
    bad = []
    inside = False
    for line in body.splitlines():
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            inside = True
        elif t.startswith(";;#ASMEND"):
            inside = False
        elif t and not t.startswith((";", ".")) and not inside and ("accvgpr" in t or re.search(r"\ba\[?\d", t)):
            bad.append("compiler AGPR use: " + t)
    if "scratch_" in body:
        bad.append(f"scratch traffic in {kname}")
    ins = [t.strip() for t in body.splitlines()]
    ins = [t.replace(",", " ").split() for t in ins if t and not t.startswith((";", "."))]
    n_dma = 0
    for i, u in enumerate(ins):
        if not (u[0].startswith("buffer_load") and u[-1] == "lds" and ins[i - 4] != ["s_nop", "4"]):
            continue
        n_dma += 1
        srd = _sgprs(u[2])
        if not srd:
            bad.append("LDS-DMA without an SGPR descriptor: " + " ".join(u))
            continue
        states = 0
        for w in reversed(ins[:i]):
            if len(w) > 1 and not w[0].startswith(_NO_DST) and w[0].startswith(("s_", "v_")) and _sgprs(w[1]) & srd:
                if w[0].startswith("v_") and states < 5:
                    bad.append(f"descriptor hazard: {' '.join(w)} {states} states before {' '.join(u)}")
                break
            states += int(w[1]) + 1 if w[0] == "s_nop" else 1
    if n_dma == 0:
        bad.append("no LDS-DMA without its own s_nop found: the audit no longer matches the kernel")
    return bad


audit_x64 = audit_asm_kernel          # the round-2 name


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
