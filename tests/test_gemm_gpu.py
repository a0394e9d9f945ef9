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


@pytest.fixture(params=["auto", "8wave", "w4", "w4_alt_order"])
def gemm_variant(request):
    """Run a cram_gemm test on each kernel: the automatic choice (bf16 with >= 2 K-tiles -> gemm_w4_kernel), the
    8-wave kernel forced (knob 0), the 4-wave kernel forced (1) and the 4-wave kernel's alternative tile order (2)."""
    from cram_amd import _lib
    prev = _lib.set_knob(_lib.KNOB_GEMM_VARIANT, {"auto": -1, "8wave": 0, "w4": 1, "w4_alt_order": 2}[request.param])
    yield request.param
    _lib.set_knob(_lib.KNOB_GEMM_VARIANT, prev)


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
def test_gemm_store_matches_fp32(gpu_device, gemm_variant, dtype, M, N, K):
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


def test_gemm_strided_rows_and_tail(gpu_device, gemm_variant):
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
def test_gemm_silu_mul_epilogue(gpu_device, gemm_variant, dtype, M, F, K):
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


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K,splits", [
    (1, 256, 512, 2), (16, 512, 1024, 8), (200, 768, 2048, 4), (256, 1536, 4096, 8), (256, 1024, 4096, 16),
    (300, 512, 14336, 14), (256, 256, 256, 1), (33, 256, 3584, 7),
])
def test_gemm_splitk_store_matches_fp32(gpu_device, dtype, M, N, K, splits):
    """Split-K form (the decode step's skinny projections): same final-rounding bar as the one-pass GEMM; a second
    launch is bit-identical (the ranges are added in range order, no atomics)."""
    x, w = _operands(M, N, K, dtype, gpu_device, 11 * M + N + K + splits)
    ws = torch.empty(ops.gemm_splitk_workspace_bytes(M, N, splits), dtype=torch.uint8, device=gpu_device)
    out = ops.gemm_splitk(x, w, splits, workspace=ws)
    again = ops.gemm_splitk(x, w, splits, workspace=ws)
    ref = x.float() @ w.float().t()
    acc_tol = 2.0 ** -22 * (x.float().abs() @ w.float().abs().t())
    torch.cuda.synchronize()
    assert torch.equal(out, again)
    d = (out.float() - ref).abs()
    assert (d <= _ulp(ref, dtype) + acc_tol).all(), f"max err {d.max().item():.3e}"
    assert (out == ref.to(dtype)).float().mean().item() >= 0.99


def test_gemm_splitk_bias_and_strided_rows(gpu_device):
    """nn.Linear with bias (Qwen2's q/k/v): out = rnd(x w^T + b); strided activation rows and output rows."""
    M, N, K = 77, 512, 1024
    x0, w = _operands(M, N, K + 64, torch.bfloat16, gpu_device, 21)
    x, w = x0[:, 64:], w[:, :K].contiguous()
    b = (torch.rand(N, generator=torch.Generator().manual_seed(3)) - 0.5).to(torch.bfloat16).to(gpu_device)
    big = torch.full((M, N + 64), 7.0, dtype=torch.bfloat16, device=gpu_device)
    out = big[:, 32:32 + N]
    ops.gemm_splitk(x, w, 4, bias=b, out=out)
    ref = x.float() @ w.float().t() + b.float()
    torch.cuda.synchronize()
    assert ((out.float() - ref).abs() <= _ulp(ref, torch.bfloat16) + 1e-5).all()
    assert (big[:, :32] == 7).all() and (big[:, 32 + N:] == 7).all()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,F,K,splits", [(1, 128, 512, 2), (256, 1024, 4096, 2), (16, 384, 3584, 7)])
def test_gemm_splitk_silu_mul_cat(gpu_device, dtype, M, F, K, splits):
    """The MLP activation on the checkpoint's own [gate; up] weight: rnd(rnd(silu(rnd(g))) * rnd(u)), the arithmetic
    of cram_silu_mul on the rounded projections; bit-identical to split-K STORE followed by cram_silu_mul."""
    x, wgu = _operands(M, 2 * F, K, dtype, gpu_device, 5 * M + F + K)
    out = ops.gemm_splitk(x, wgu, splits, ops.GEMM_SILU_MUL_CAT)
    unfused = ops.silu_mul(ops.gemm_splitk(x, wgu, splits), F)
    ref = x.float() @ wgu.float().t()
    exp = _silu_mul_expected(ref[:, :F], ref[:, F:], dtype)
    torch.cuda.synchronize()
    assert out.shape == (M, F)
    assert torch.equal(out, unfused)
    d = (out.float() - exp.float()).abs()
    # a 1-ulp difference of each rounded projection propagates through silu and the product: every element within
    # 4 ulp, >= 99 % within 1 (M = 1 has only 128 elements)
    assert (d <= 4 * _ulp(exp.float(), dtype) + 1e-6).all(), float((d / _ulp(exp.float(), dtype)).max())
    assert (d <= _ulp(exp.float(), dtype) + 1e-6).float().mean().item() >= 0.99


def test_engine_fused_mlp_matches_library_pair(gpu_device):
    """CrAMEngine.mlp at sweep row counts (gate/up on gemm_w4_kernel with the SiLU-mul epilogue, the interleaved
    weight built from the checkpoint's [gate; up]) == hipBLASLt gate/up + cram_silu_mul within the bf16 noise of two
    GEMM accumulation orders; an in-place weight edit (tests/planted.py does this) rebuilds the interleaved copy."""
    from cram_amd import engine as E
    sp = E.ModelSpec(1, 1024, 8, 2, 128, 1536, 1000, 1e-5, False)
    eng = E.CrAMEngine.random(sp, gpu_device, seed=11, std=0.03)
    lw = eng.layers[0]
    x = (torch.randn(4608, sp.hidden, device=gpu_device, generator=torch.Generator(device=gpu_device).manual_seed(2))
         ).to(torch.bfloat16)
    assert eng._fused_mlp_ok(x)
    fused = eng.mlp(x, lw)
    prev = E.FUSED_MLP
    E.FUSED_MLP = False
    try:
        lib = eng.mlp(x, lw)
    finally:
        E.FUSED_MLP = prev
    d = (fused.float() - lib.float()).abs()
    scale = lib.float().abs().mean().item()
    assert d.max().item() <= 0.05 * lib.float().abs().max().item() and d.mean().item() <= 0.01 * scale, (d.max(), scale)
    lw.wgu[:, :7] = 0                                            # in place: the interleaved copy must follow
    E.FUSED_MLP = False
    try:
        lib2 = eng.mlp(x, lw)
    finally:
        E.FUSED_MLP = prev
    fused2 = eng.mlp(x, lw)
    d2 = (fused2.float() - lib2.float()).abs()
    assert d2.mean().item() <= 0.01 * lib2.float().abs().mean().item()
    assert not torch.equal(fused2, fused)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (77, 512, 128), (300, 768, 4096), (4097, 1536, 4096),
                                   (513, 256, 14336)])
def test_gemm_residual_epilogue(gpu_device, gemm_variant, dtype, M, N, K):
    """cram_gemm_residual (o_proj / down_proj with the decoder layer's residual add): out = rnd(res + rnd(acc)),
    bit-identical to the same kernel's plain GEMM followed by a model-dtype add (HF's `residual + hidden_states`);
    in place (out = res) gives the same bits."""
    x, w = _operands(M, N, K, dtype, gpu_device, 13 * M + N + K)
    g = torch.Generator(device="cpu").manual_seed(M + K)
    res = ((torch.rand(M, N, generator=g) * 8 - 4).to(dtype)).to(gpu_device)
    out = ops.gemm(x, w, residual=res)
    exp = ops.gemm(x, w) + res                   # bf16 / fp16 add: fp32 sum of the two, rounded once
    inplace = res.clone()
    ops.gemm(x, w, residual=inplace, out=inplace)
    ref = x.float() @ w.float().t() + res.float()
    torch.cuda.synchronize()
    assert out.shape == (M, N) and torch.isfinite(out.float()).all()
    assert torch.equal(out, exp)
    assert torch.equal(inplace, out)
    acc_tol = 2.0 ** -22 * (x.float().abs() @ w.float().abs().t())
    d = (out.float() - ref).abs()
    # two roundings (the product, then the sum): within 1 ulp of the product plus 1 ulp of the sum
    bar = _ulp(ref - res.float(), dtype) + _ulp(ref, dtype) + acc_tol
    assert (d <= bar).all(), f"max err {d.max().item():.3e}"


def test_gemm_residual_strided_rows_and_tail(gpu_device, gemm_variant):
    """Residual and output as views into wider buffers, M not a multiple of the 256-row tile: nothing outside the
    [M][N] output view is written."""
    M, N, K = 333, 512, 256
    x, w = _operands(M, N, K, torch.bfloat16, gpu_device, 17)
    rbig = torch.randn(M, N + 64, device=gpu_device).to(torch.bfloat16)
    res = rbig[:, 64:]
    big = torch.full((M + 7, N + 128), 7.0, dtype=torch.bfloat16, device=gpu_device)
    out = big[:M, 64:64 + N]
    ops.gemm(x, w, out=out, residual=res)
    exp = ops.gemm(x, w) + res
    torch.cuda.synchronize()
    assert torch.equal(out, exp)
    assert (big[M:] == 7).all() and (big[:M, :64] == 7).all() and (big[:M, 64 + N:] == 7).all()


def test_engine_fused_residual_layer_matches_deferred_add(gpu_device):
    """CrAMEngine.o_proj_norm / mlp_residual at sweep row counts (residual adds in the o_proj / down_proj epilogues)
    == the deferred-add path (F.linear, the add inside the next RMSNorm) within the bf16 noise of two GEMM
    accumulation orders; with the same GEMM on both sides the layer output is bit-identical."""
    from cram_amd import engine as E
    sp = E.ModelSpec(1, 1024, 8, 2, 128, 1536, 1000, 1e-5, False)
    eng = E.CrAMEngine.random(sp, gpu_device, seed=12, std=0.03)
    lw = eng.layers[0]
    gen = torch.Generator(device=gpu_device).manual_seed(4)
    a = torch.randn(4608, sp.q_size, device=gpu_device, generator=gen).to(torch.bfloat16)
    h = torch.randn(4608, sp.hidden, device=gpu_device, generator=gen).to(torch.bfloat16)
    assert eng._fused_residual_ok(a)
    h2, x2 = eng.o_proj_norm(a, lw, h)
    hout, m = eng.mlp_residual(x2, lw, h2)
    assert m is None
    # the same arithmetic with the add outside the GEMMs (cram_gemm both times: identical accumulation)
    h2_ref, x2_ref = ops.rmsnorm(ops.gemm(a, lw.wo), lw.ln2, sp.eps, residual=h)
    act = ops.gemm(x2_ref, eng._gate_up_interleaved(lw), ops.GEMM_SILU_MUL)
    hout_ref = h2_ref + ops.gemm(act, lw.wd)
    prev = E.FUSED_RESIDUAL
    E.FUSED_RESIDUAL = False
    try:
        h2_lib, x2_lib = eng.o_proj_norm(a, lw, h)
        hl, ml = eng.mlp_residual(x2_lib, lw, h2_lib)
    finally:
        E.FUSED_RESIDUAL = prev
    torch.cuda.synchronize()
    assert torch.equal(h2, h2_ref) and torch.equal(x2, x2_ref) and torch.equal(hout, hout_ref)
    lib = hl + ml
    d = (hout.float() - lib.float()).abs()
    scale = lib.float().abs().mean().item()
    assert d.max().item() <= 0.05 * lib.float().abs().max().item() and d.mean().item() <= 0.01 * scale, (d.max(), scale)


def _rope_tables(P, d, dev, theta=500000.0, dtype=torch.bfloat16):
    inv = 1.0 / theta ** (torch.arange(0, d, 2, dtype=torch.float32) / d)
    f = torch.arange(P, dtype=torch.float32)[:, None] * inv[None]
    emb = torch.cat((f, f), -1)
    return emb.cos().to(dtype).to(dev), emb.sin().to(dtype).to(dev)


HQ, HKV, HD = 32, 8, 128


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K", [256, 4096])
def test_gemm_rope_inplace_equals_gemm_then_rope(gpu_device, K, dtype):
    """cram_gemm_rope without kout (the sweep's suffix layers when no prefix is shared): bit-identical to the same
    kernel's plain GEMM followed by cram_rope_inplace over the q and k heads; v heads as computed; GEMM padding rows
    [rows, M) read table row 0 and are never compared."""
    B, T = 3, 1000
    rows, M = B * T, 3072
    x, w = _operands(M, (HQ + 2 * HKV) * HD, K, dtype, gpu_device, 41 + K)
    cos, sin = _rope_tables(T, HD, gpu_device, dtype=dtype)
    out = ops.gemm_rope(x, w, HQ, HKV, HD, cos, sin, T, rows=rows)
    ref = ops.gemm(x, w)
    ops.rope_inplace(ref[:rows], HQ + HKV, HD, cos, sin, T=T)
    torch.cuda.synchronize()
    assert torch.equal(out[:rows], ref[:rows])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gemm_rope_bias(gpu_device, dtype):
    """cram_gemm_rope with Qwen2's q/k/v bias: the projection is rnd(acc + bias) (F.linear's rounding) before RoPE.
    With identity tables (cos 1, sin 0) the result is that projection itself: within the final-rounding bar of the
    float32 product plus the bias; with real tables it equals RoPE applied to it (cram_rope_inplace)."""
    B, T, K = 2, 700, 512
    rows, M = B * T, 1536
    N = (HQ + 2 * HKV) * HD
    x, w = _operands(M, N, K, dtype, gpu_device, 53)
    b = (torch.rand(N, generator=torch.Generator().manual_seed(4)) - 0.5).to(dtype).to(gpu_device)
    one = torch.ones(T, HD, dtype=dtype, device=gpu_device)
    zero = torch.zeros(T, HD, dtype=dtype, device=gpu_device)
    proj = ops.gemm_rope(x, w, HQ, HKV, HD, one, zero, T, rows=rows, bias=b)
    ref = x.float() @ w.float().t() + b.float()
    acc_tol = 2.0 ** -22 * (x.float().abs() @ w.float().abs().t())
    cos, sin = _rope_tables(T, HD, gpu_device, dtype=dtype)
    out = ops.gemm_rope(x, w, HQ, HKV, HD, cos, sin, T, rows=rows, bias=b)
    exp = proj.clone()
    ops.rope_inplace(exp[:rows], HQ + HKV, HD, cos, sin, T=T)
    torch.cuda.synchronize()
    d = (proj[:rows].float() - ref[:rows]).abs()
    assert (d <= _ulp(ref[:rows], dtype) + acc_tol[:rows]).all(), float(d.max())
    assert torch.equal(out[:rows], exp[:rows])


def test_gemm_rope_split_behind_prefix(gpu_device):
    """The sweep's layer_rows with a shared prefix: q rotated in place, k rotated into and v copied into the
    [B, p0 + T] key / value buffers behind the prefix at table rows pos = p0 + t; == GEMM + cram_rope_split, the
    prefix rows untouched, nothing written for the GEMM padding rows."""
    B, T, p0 = 5, 700, 25
    rows = B * T
    M = 3584
    x, w = _operands(M, (HQ + 2 * HKV) * HD, 512, torch.bfloat16, gpu_device, 43)
    cos, sin = _rope_tables(p0 + T, HD, gpu_device)
    pos = (torch.arange(T, device=gpu_device, dtype=torch.int64) + p0).repeat(B)
    g = torch.Generator(device="cpu").manual_seed(2)
    k0 = torch.randn(B, p0 + T + 3, HKV, HD, generator=g).to(torch.bfloat16).to(gpu_device)
    v0 = torch.randn(B, p0 + T + 3, HKV, HD, generator=g).to(torch.bfloat16).to(gpu_device)
    k, v, kr, vr = k0.clone(), v0.clone(), k0.clone(), v0.clone()
    out = ops.gemm_rope(x, w, HQ, HKV, HD, cos, sin, T, rows=rows, kout=k, vout=v, row0=p0, pos=pos)
    ref = ops.gemm(x, w)
    ops.rope_split(ref[:rows], HQ, HKV, HD, cos, sin, T, kr, vr, p0, pos=pos)
    torch.cuda.synchronize()
    assert torch.equal(out[:rows, :HQ * HD], ref[:rows, :HQ * HD])
    assert torch.equal(k, kr) and torch.equal(v, vr)
    assert torch.equal(k[:, :p0], k0[:, :p0]) and torch.equal(k[:, p0 + T:], k0[:, p0 + T:])


def test_gemm_rope_split_into_cache_keep_k(gpu_device):
    """The packed decode prefill: ragged sequences packed row after row, K/V scattered into the cache
    ([B, Hkv, S, d] seen as [B, S, Hkv, d]) at (dst_b[m], pos[m]); keep_k leaves the rotated k and v in the buffer
    for the varlen attention; == GEMM + cram_rope_split(keep_k)."""
    lens = [300, 1, 777, 64, 1000]
    total = sum(lens)
    M = 2304
    S = 1024
    x, w = _operands(M, (HQ + 2 * HKV) * HD, 256, torch.bfloat16, gpu_device, 47)
    cos, sin = _rope_tables(S, HD, gpu_device)
    pos = torch.cat([torch.arange(n, dtype=torch.long) for n in lens]).to(gpu_device)
    bidx = torch.cat([torch.full((n,), b, dtype=torch.long) for b, n in enumerate(lens)]).to(gpu_device)
    kc = torch.zeros(len(lens), HKV, S, HD, dtype=torch.bfloat16, device=gpu_device)
    vc = torch.zeros_like(kc)
    kcr, vcr = kc.clone(), vc.clone()
    out = ops.gemm_rope(x, w, HQ, HKV, HD, cos, sin, 1, rows=total, kout=kc.transpose(1, 2),
                        vout=vc.transpose(1, 2), row0=0, pos=pos, dst_b=bidx, keep_k=True)
    ref = ops.gemm(x, w)
    ops.rope_split(ref[:total], HQ, HKV, HD, cos, sin, 1, kcr.transpose(1, 2), vcr.transpose(1, 2), 0, pos=pos,
                   dst_b=bidx, keep_k=True)
    torch.cuda.synchronize()
    assert torch.equal(out[:total], ref[:total])
    assert torch.equal(kc, kcr) and torch.equal(vc, vcr)


@pytest.mark.parametrize("qkv_bias", [False, True])
def test_engine_fused_qkv_layer_matches_library_path(gpu_device, qkv_bias):
    """CrAMEngine.layer_rows at sweep row counts with RoPE in the q/k/v GEMM's epilogue == the library path
    (hipBLASLt + cram_rope_split) within the bf16 noise of two GEMM accumulation orders, with and without a shared
    prefix; Llama (no bias) and Qwen2 (q/k/v bias in the epilogue)."""
    from cram_amd import engine as E
    sp = E.ModelSpec(2, 1024, 8, 2, 128, 1536, 1000, 1e-5, qkv_bias)
    eng = E.CrAMEngine.random(sp, gpu_device, seed=13, std=0.03)
    B, T, p0 = 9, 500, 20
    gen = torch.Generator(device=gpu_device).manual_seed(5)
    h = torch.randn(B * T, sp.hidden, device=gpu_device, generator=gen).to(torch.bfloat16)
    cos, sin = eng.rope_tables(p0 + T)
    k0 = torch.randn(1, p0, sp.num_kv_heads, sp.head_dim, device=gpu_device, generator=gen).to(torch.bfloat16)
    v0 = torch.randn_like(k0)
    assert eng._fused_qkv_ok(h, eng.layers[1])
    for pre in (None, (k0, v0)):
        fused = eng.layer_rows(h, B, T, 1, cos, sin, prefix=pre)
        prev = E.FUSED_QKV
        E.FUSED_QKV = False
        try:
            lib = eng.layer_rows(h, B, T, 1, cos, sin, prefix=pre)
        finally:
            E.FUSED_QKV = prev
        torch.cuda.synchronize()
        of = fused[0] if fused[1] is None else fused[0] + fused[1]
        ol = lib[0] if lib[1] is None else lib[0] + lib[1]
        d = (of.float() - ol.float()).abs()
        scale = ol.float().abs().mean().item()
        assert d.max().item() <= 0.05 * ol.float().abs().max().item() and d.mean().item() <= 0.01 * scale


@pytest.mark.parametrize("M,N,K,splits", [(512, 4096, 4096, 8), (77, 512, 14336, 4), (256, 768, 1024, 2)])
def test_gemm_splitk_residual(gpu_device, M, N, K, splits):
    """cram_gemm_splitk_residual: rnd(res + rnd(sum over the K ranges)), bit-identical to split-K STORE followed by a
    model-dtype add, in place too."""
    x, w = _operands(M, N, K, torch.bfloat16, gpu_device, 19 * M + K)
    res = (torch.randn(M, N, generator=torch.Generator().manual_seed(M)) * 2).to(torch.bfloat16).to(gpu_device)
    out = ops.gemm_splitk(x, w, splits, residual=res)
    exp = ops.gemm_splitk(x, w, splits) + res
    inplace = res.clone()
    ops.gemm_splitk(x, w, splits, residual=inplace, out=inplace)
    torch.cuda.synchronize()
    assert torch.equal(out, exp) and torch.equal(inplace, out)


@pytest.mark.parametrize("K", [4096, 14336])
def test_engine_residual_gemm_tail_split(gpu_device, K):
    """CrAMEngine._gemm_residual at the sweep's row count M = 29,184 (N = 4096: 1,824 tiles = 7 waves of 256 + 32):
    rows past the last whole wave go through split-K.  Rows in the whole waves are bit-identical to the one-launch
    residual GEMM, tail rows to split-K + add; all within the final-rounding bar of the float32 product."""
    from cram_amd import engine as E
    sp = E.ModelSpec(1, 1024, 8, 2, 128, 1536, 1000, 1e-5, False)
    eng = E.CrAMEngine.random(sp, gpu_device, seed=3, std=0.03)
    M, N = 29184, 4096
    x, w = _operands(M, N, K, torch.bfloat16, gpu_device, 23 + K)
    h = (torch.randn(M, N, generator=torch.Generator().manual_seed(9)) * 2).to(torch.bfloat16).to(gpu_device)
    out = eng._gemm_residual(x, w, h)
    one = ops.gemm(x, w, residual=h)
    Mm = 28672                                    # 7 waves x 256 tiles / 16 column tiles = 112 row tiles
    torch.cuda.synchronize()
    assert torch.equal(out[:Mm], one[:Mm])
    assert not torch.equal(out[Mm:], one[Mm:])    # the tail did go through the other kernel
    for s in (8,):
        assert torch.equal(out[Mm:], ops.gemm_splitk(x[Mm:], w, s) + h[Mm:])
    rows = slice(Mm - 64, M)
    ref = x[rows].float() @ w.float().t()
    acc_tol = 2.0 ** -22 * (x[rows].float().abs() @ w.float().abs().t())
    d = (out[rows].float() - (ref + h[rows].float())).abs()
    bar = _ulp(ref, torch.bfloat16) + _ulp(ref + h[rows].float(), torch.bfloat16) + acc_tol
    assert (d <= bar).all(), float(d.max())


# ---------------------------------------------------------------------------------------------------------------
# cram_gemm_small: the decode step's projections (128 x 128 tiles, four-deep ring, optional K split)
# ---------------------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K,splits", [
    (1, 128, 64, 1), (5, 256, 192, 1), (129, 384, 4096, 1), (500, 6144, 4096, 1), (512, 4096, 4096, 2),
    (128, 1024, 14336, 4), (200, 768, 3584, 7), (77, 512, 128, 2), (256, 640, 320, 5),
])
def test_gemm_small_matches_fp32(gpu_device, dtype, M, N, K, splits):
    """Every tile / ring / K-split / tail path: single-tile K ranges (K = 64), ranges shorter than the ring
    (2-3 K-tiles), the steady state, ragged M (rows past M read as zeros, never stored)."""
    x, w = _operands(M, N, K, dtype, gpu_device, 3 * M + N + K + splits)
    out = torch.full((M + 3, N), 7.0, dtype=dtype, device=gpu_device)
    ops.gemm_small(x, w, splits, out=out[:M])
    ref = x.float() @ w.float().t()
    acc_tol = 2.0 ** -22 * (x.float().abs() @ w.float().abs().t())
    torch.cuda.synchronize()
    d = (out[:M].float() - ref).abs()
    assert (d <= _ulp(ref, dtype) + acc_tol).all(), f"max err {d.max().item():.3e}"
    assert (out[:M] == ref.to(dtype)).float().mean().item() >= 0.99
    assert (out[M:] == 7).all()


@pytest.mark.parametrize("splits", [1, 4])
def test_gemm_small_bias_and_silu_mul(gpu_device, splits):
    """F.linear with a bias (Qwen2's q/k/v: rnd(acc + b), the split-K combine's rule too) and the SiLU-mul epilogue
    on the interleaved gate/up weight == the same GEMM stored, then cram_silu_mul (bit for bit, either split)."""
    M, N, K, F = 300, 1024, 2048, 1024
    x, w = _operands(M, N, K, torch.bfloat16, gpu_device, 11)
    b = (torch.randn(N, device=gpu_device) * 0.5).to(torch.bfloat16)
    out = ops.gemm_small(x, w, splits, bias=b)
    ref = (x.float() @ w.float().t() + b.float())
    torch.cuda.synchronize()
    assert ((out.float() - ref).abs() <= _ulp(ref, torch.bfloat16) + 1e-5).all()
    xg, wgu = _operands(M, 2 * F, K, torch.bfloat16, gpu_device, 12)
    wil = ops.interleave_gate_up(wgu, F)
    act = ops.gemm_small(xg, wil, splits, ops.GEMM_SILU_MUL)
    plain = ops.gemm_small(xg, wgu, splits)
    torch.cuda.synchronize()
    assert torch.equal(act, ops.silu_mul(plain, F))


def test_gemm_small_rejects_bad_arguments(gpu_device):
    from cram_amd import _lib
    x, w = _operands(64, 256, 256, torch.bfloat16, gpu_device, 1)
    with pytest.raises(RuntimeError, match="CRAM error -2"):
        ops.gemm_small(x, w[:200])                    # N % 128
    with pytest.raises(RuntimeError, match="CRAM error -2"):
        ops.gemm_small(x, w, 3)                       # K % (64 * splits)
    L = _lib.load()
    o = torch.empty(64, 256, dtype=torch.bfloat16, device=gpu_device)
    code = L.cram_gemm_small(x.data_ptr(), 256, w.data_ptr(), 256, None, o.data_ptr(), 256, 64, 256, 256, 2,
                             ops.GEMM_STORE, None, 0, 0, None)
    assert code == -5                                 # CRAM_ERR_WORKSPACE: splits > 1 without a workspace
