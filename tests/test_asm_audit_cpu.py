"""prefill_x32_kernel owns accumulator registers by name (O = a[0:63], Q = a[64:95]), and so does gemm_w4_kernel
(all of a[0:255]); hipcc knows nothing of that ownership, so a compiler spill or copy into the AGPR file would silently
corrupt O, Q or the GEMM accumulators.  cram_amd.build runs the audit
(cram_amd.build.audit_asm_kernel) on the device assembly of every build it makes and refuses to install a library that fails
it; this CPU test re-checks the assembly of the current build: no v_accvgpr_* instruction or AGPR operand outside the
kernel's own inline-asm statements, no scratch traffic, and 5 wait states between any VALU write of an LDS-DMA
descriptor SGPR and the DMA (the kernel's DMA pieces after the first of a tile carry no s_nop of their own)."""
import os
import shutil

import pytest

from cram_amd import build

pytestmark = pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                                reason="hipcc not available")


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    """The device assembly of the current sources: the last build's saved .s when it matches them, else a
    device-only compile into a temporary directory (the installed library is never rebuilt or replaced here)."""
    return build.device_asm(tmp_path_factory.mktemp("asm"))


def test_every_register_owning_instantiation_is_audited(asm):
    """The audited list comes from the assembly: every epilogue (store, SiLU-mul, split-K partial, residual, RoPE) of
    gemm_w4_kernel in both element types, and prefill_x32_kernel."""
    names = build.asm_kernels(asm)
    w4 = [n for n in names if "gemm_w4_kernel" in n]
    for epi in ("Li0E", "Li1E", "Li100E", "Li101E", "Li102E"):
        for dt in ("DF16b", "DF16_"):
            assert any(dt + epi in n for n in w4), (dt, epi, w4)
    assert any("prefill_x32_kernel" in n for n in names)


def test_asm_kernel_register_ownership_and_dma_hazards(asm):
    bad = {k: build.audit_asm_kernel(asm, k) for k in build.asm_kernels(asm)}
    assert {k: v for k, v in bad.items() if v} == {}


def test_audit_catches_a_compiler_agpr_and_scratch_traffic(asm):
    for kname in build.asm_kernels(asm):
        body = build.kernel_body(asm, kname)
        assert build.audit_asm_kernel(asm.replace(body, body + "\n\tv_accvgpr_write_b32 a5, v1\n", 1), kname), kname
        assert any("scratch" in b for b in build.audit_asm_kernel(
            asm.replace(body, body + "\n\tscratch_store_dword v0, v1, off\n", 1), kname)), kname
