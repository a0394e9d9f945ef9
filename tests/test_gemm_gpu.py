"""cram_gemm (hand-written CDNA4 MFMA projection GEMM, cram_amd/csrc/cram_gemm.hip) vs a float32 PyTorch reference.

The GEMM replaces F.linear for the LlamaMLP gate/up projection and fuses its activation (the reference's
nn.Linear + act_fn inside every hooked forward: /root/reference/utils/re_weighting.py:158,170 -> transformers
LlamaMLP).  bf16 / fp16 in and out, fp32 accumulation in a different order than any reference: the bar is the
final rounding — every element within 1 ulp of the model-dtype rounding of the float32 product (and >= 99 % of
them equal to it); the SiLU-mul epilogue within 1 ulp of rnd(rnd(silu(rnd(g))) * rnd(u)) on >= 99.5 % of the
elements (cram_silu_mul's bar), and bit-identical to the unfused GEMM + cram_silu_mul on the same weight.
"""
import pytest
import torch

from cram_amd import ops

pytestmark = pytest.mark.gpu


def _ulp(x: torch.Tensor, dtype) -> torch.Tensor:
    """ulp of the model dtype at |x| (float32 tensor)."""
    mant = 7 if dtype == torch.bfloat16 else 10
    e = torch.floor(torch.log2(x.abs().clamp_min(2.0 ** -14)))
    return torch.exp2(e - mant)


def _operands(M, N, K, dtype, dev, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(dtype).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) * (K ** -0.5)).to(dtype).to(dev)
    return x, w


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [
    (1, 256, 64), (77, 512, 128), (256, 256, 192), (300, 768, 4096), (1000, 1024, 320), (2048, 2048, 1024),
    (4097, 1536, 4096), (513, 256, 14336),
])
def test_gemm_store_matches_fp32(gpu_device, dtype, M, N, K):
    x, w = _operands(M, N, K, dtype, gpu_device, 7 * M + N + K)
    out = ops.gemm(x, w)
    ref = x.float() @ w.float().t()
    # two float32 sums of the same K products in different orders differ by up to ~2^-22 of the sum of |products|
    acc_tol = 2.0 ** -22 * (x.float().abs() @ w.float().abs().t())
    torch.cuda.synchronize()
    assert out.shape == (M, N) and out.dtype == dtype
    d = (out.float() - ref).abs()
    assert torch.isfinite(out.float()).all()
    assert (d <= _ulp(ref, dtype) + acc_tol).all(), f"max err {d.max().item():.3e}"
    exact = (out == ref.to(dtype)).float().mean().item()
    assert exact >= 0.99, exact


def test_gemm_strided_rows_and_tail(gpu_device):
    """Row strides wider than K (views into fused buffers) and M not a multiple of the 256-row tile; rows past M
    stay untouched."""
    M, N, K = 333, 512, 256
    x0, w0 = _operands(M, N, K + 64, torch.bfloat16, gpu_device, 5)
    x, w = x0[:, 32:32 + K], w0[:, :K]
    big = torch.full((M + 7, N + 128), 7.0, dtype=torch.bfloat16, device=gpu_device)
    out = big[:M, 64:64 + N]
    ops.gemm(x, w, out=out)
    ref = x.float() @ w.float().t()
    torch.cuda.synchronize()
    assert ((out.float() - ref).abs() <= _ulp(ref, torch.bfloat16) + 1e-6).all()
    assert (big[M:] == 7).all() and (big[:M, :64] == 7).all() and (big[:M, 64 + N:] == 7).all()


def _silu_mul_expected(g32, u32, dtype):
    g = g32.to(dtype).float()
    s = torch.nn.functional.silu(g).to(dtype).float()
    return (s * u32.to(dtype).float()).to(dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,F,K", [(1, 128, 64), (300, 256, 512), (1111, 384, 4096), (2048, 1024, 1024)])
def test_gemm_silu_mul_epilogue(gpu_device, dtype, M, F, K):
    x, wgu = _operands(M, 2 * F, K, dtype, gpu_device, 3 * M + F + K)
    wil = ops.interleave_gate_up(wgu, F)
    out = ops.gemm(x, wil, ops.GEMM_SILU_MUL)
    ref = x.float() @ wgu.float().t()
    exp = _silu_mul_expected(ref[:, :F], ref[:, F:], dtype)
    # the unfused pipeline on the same GEMM: identical accumulation order per element -> bit-identical
    unfused = ops.silu_mul(ops.gemm(x, wgu), F)
    torch.cuda.synchronize()
    assert out.shape == (M, F)
    assert torch.equal(out, unfused)
    d = (out.float() - exp.float()).abs()
    within = (d <= _ulp(exp.float(), dtype) + 1e-6).float().mean().item()
    assert within >= 0.995, within


def test_interleave_gate_up_layout():
    F, K = 64, 8
    wgu = torch.arange(2 * F, dtype=torch.float32)[:, None].expand(2 * F, K).contiguous()
    wil = ops.interleave_gate_up(wgu, F)[:, 0].long().tolist()
    assert wil[:32] == list(range(32)) and wil[32:64] == list(range(F, F + 32))
    assert wil[64:96] == list(range(32, 64)) and wil[96:] == list(range(F + 32, 2 * F))
