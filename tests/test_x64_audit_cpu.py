"""prefill_x64_kernel owns accumulator registers by name (O = a[0:127], Q = a[128:191]); hipcc knows nothing of that
ownership, so a compiler spill or copy into the AGPR file would silently corrupt O or Q.  This CPU test compiles the
library for gfx950 to assembly and requires that no v_accvgpr_* instruction or AGPR operand appears outside the kernel's
own inline-asm statements, and that the kernel has no scratch traffic (tools/agpr_audit.py does the same by hand)."""
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


def test_x64_kernel_uses_no_compiler_agprs(tmp_path):
    out = tmp_path / "cram_attn.s"
    cmd = [build._hipcc(), f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "--cuda-device-only", "-S",
           "-I", str(build.REPO_DIR / "include"), str(build.CSRC / "cram_attn.hip"), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True)
    body = _kernel_body(out.read_text(), "prefill_x64_kernel")
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
