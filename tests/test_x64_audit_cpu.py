"""prefill_x64_kernel owns accumulator registers by name (O = a[0:127], Q = a[128:191]); hipcc knows nothing of that
ownership, so a compiler spill or copy into the AGPR file would silently corrupt O or Q.  This CPU test compiles the
library for gfx950 to assembly and requires that no v_accvgpr_* instruction or AGPR operand appears outside the kernel's
own inline-asm statements, and that the kernel has no scratch traffic (tools/agpr_audit.py does the same by hand).
The kernel's LDS-DMA pieces after the first of a tile carry no s_nop of their own, so the test also walks back from
every LDS-DMA and requires 5 wait states between any VALU write of an SGPR of its descriptor and the DMA."""
import os
import re
import shutil
import subprocess

import pytest

from cram_amd import build

pytestmark = pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                                reason="hipcc not available")


def _kernel_body(asm, name):
    m = re.search(r"^(_Z\w*" + name + r"\w*):", asm, re.M)
    assert m, f"kernel {name} not found in the assembly"
    return asm[m.end(): asm.find(".Lfunc_end", m.end())]


@pytest.fixture(scope="module")
def x64_body(tmp_path_factory):
    out = tmp_path_factory.mktemp("x64") / "cram_attn.s"
    cmd = [build._hipcc(), f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "--cuda-device-only", "-S",
           "-I", str(build.REPO_DIR / "include"), str(build.CSRC / "cram_attn.hip"), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True)
    return _kernel_body(out.read_text(), "prefill_x64_kernel")


def _sgprs(op):
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", op)
    return {int(m.group(1))} if m else set()


_NO_DST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_barrier", "s_setprio", "s_endpgm")


def test_x64_dma_descriptor_hazards(x64_body):
    # every LDS-DMA without its own s_nop 4: walking back in program order, the latest write of any SGPR of its
    # descriptor is scalar (no hazard) or a VALU write at least 5 wait states earlier
    ins = [t.strip() for t in x64_body.splitlines()]
    ins = [t.replace(",", " ").split() for t in ins if t and not t.startswith((";", "."))]
    bare = 0
    for i, u in enumerate(ins):
        if not (u[0].startswith("buffer_load") and u[-1] == "lds" and ins[i - 4] != ["s_nop", "4"]):
            continue
        bare += 1
        srd = _sgprs(u[2])
        assert srd, u
        states = 0
        for w in reversed(ins[:i]):
            if len(w) > 1 and not w[0].startswith(_NO_DST) and (w[0].startswith(("s_", "v_"))) and _sgprs(w[1]) & srd:
                assert not w[0].startswith("v_") or states >= 5, f"{' '.join(w)} {states} states before {' '.join(u)}"
                break
            states += int(w[1]) + 1 if w[0] == "s_nop" else 1
    assert bare > 0


def test_x64_kernel_uses_no_compiler_agprs(x64_body):
    body = x64_body
    inside, bad = False, []
    for line in body.splitlines():
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            inside = True
        elif t.startswith(";;#ASMEND"):
            inside = False
        elif t and not t.startswith((";", ".")) and not inside and ("accvgpr" in t or re.search(r"\ba\[?\d", t)):
            bad.append(t)
    assert not bad, f"hipcc touches the kernel-owned accumulator file: {bad[:5]}"
    assert "scratch_" not in body
