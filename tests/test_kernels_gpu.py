"""Kernel parity: HIP attention / answer-logit kernels vs the CPU oracle (float64).

The oracle builds the reference hook's dense [1, H, T, S] mask
(re_weighting.py:36-61) and runs softmax attention in float64; the HIP kernels
take the O(S) bias vector instead.  bf16 inputs, fp32 accumulation, bf16 output:
tolerance |err| <= 2e-2 + 2e-2 |ref| elementwise and mean |err| <= 2e-3.
"""
import math

import pytest
import torch

from oracle import hook_ref

pytestmark = pytest.mark.gpu

ATOL, RTOL, MEAN_TOL = 2e-2, 2e-2, 2e-3


def _bias_inputs(B, Hq, S, W, gen, spans_scores=((3, 40, 0.1), (41, 90, 0.0), (91, 150, 1.0), (151, 200, 0.5))):
    w = torch.ones((B, W), dtype=torch.float16)
    for (a, b, sc) in spans_scores:
        if a < W:
            w[:, a:min(b, W - 1) + 1] = sc
    lw = hook_ref.log_weight(w)                        # fp16 log, as the hook computes it
    bias = lw.to(torch.bfloat16).float()               # the value the hook writes (bf16 model)
    heads = [sorted(torch.randperm(Hq, generator=gen)[: max(1, Hq // 2)].tolist()) for _ in range(B)]
    enable = torch.zeros((B, Hq), dtype=torch.uint8)
    for b, hs in enumerate(heads):
        enable[b, hs] = 1
    return lw, bias, enable, heads


def _check(out, ref):
    out = out.double().cpu()
    assert torch.isfinite(out).all()
    err = (out - ref).abs()
    bad = err > ATOL + RTOL * ref.abs()
    assert not bad.any(), f"max err {err.max().item():.3e} at {bad.nonzero()[0].tolist()}"
    assert err.mean().item() < MEAN_TOL, f"mean err {err.mean().item():.3e}"


@pytest.mark.parametrize("B,Hq,Hkv,T,d", [
    (1, 4, 1, 1, 128), (1, 4, 2, 17, 128), (2, 8, 2, 128, 128), (1, 4, 4, 300, 128),
    (1, 8, 2, 900, 128), (1, 7, 1, 257, 128), (2, 4, 1, 200, 64), (1, 32, 8, 130, 128),
])
@pytest.mark.parametrize("biased", [False, True])
def test_prefill_matches_oracle(gpu_device, prefill_variant, B, Hq, Hkv, T, d, biased):
    gen = torch.Generator().manual_seed(1000 * T + 10 * Hq + d + biased)
    S = T
    # q laid out like transformers' transposed view: physical [B, T, Hq, d]
    q = torch.randn(B, T, Hq, d, generator=gen).to(torch.bfloat16).transpose(1, 2)
    k = torch.randn(B, Hkv, S, d, generator=gen).to(torch.bfloat16)
    v = torch.randn(B, Hkv, S, d, generator=gen).to(torch.bfloat16)
    scale = 1.0 / math.sqrt(d)
    W = max(1, S - 3)
    if biased:
        lw, bias, enable, heads = _bias_inputs(B, Hq, S, W, gen)
    else:
        lw = bias = enable = heads = None
    ref = hook_ref.biased_attention_ref(q, k, v, lw, heads, scale)
    from cram_amd import ops
    dev = gpu_device
    out = ops.attn_prefill(q.to(dev), k.to(dev), v.to(dev), scale=scale,
                           bias=None if bias is None else bias.to(dev),
                           enable=None if enable is None else enable.to(dev), W=W if biased else 0)
    torch.cuda.synchronize()
    _check(out, ref)


def test_prefill_query_offset(gpu_device, prefill_variant):
    """q_len < S (queries start at q_pos0 = S - Tq), as in chunked prefill / cached suffix."""
    gen = torch.Generator().manual_seed(7)
    B, Hq, Hkv, S, T, d = 1, 8, 2, 333, 45, 128
    q = torch.randn(B, Hq, T, d, generator=gen).to(torch.bfloat16)
    k = torch.randn(B, Hkv, S, d, generator=gen).to(torch.bfloat16)
    v = torch.randn(B, Hkv, S, d, generator=gen).to(torch.bfloat16)
    lw, bias, enable, heads = _bias_inputs(B, Hq, S, 250, gen)
    ref = hook_ref.biased_attention_ref(q, k, v, lw, heads, d ** -0.5)
    from cram_amd import ops
    dev = gpu_device
    out = ops.attn_prefill(q.to(dev), k.to(dev), v.to(dev), scale=d ** -0.5, bias=bias.to(dev),
                           enable=enable.to(dev), W=250)
    torch.cuda.synchronize()
    _check(out, ref)


@pytest.mark.parametrize("B,Hq,Hkv,S,d,splits", [
    (1, 4, 1, 1, 128, 1), (1, 32, 8, 900, 128, 1), (3, 32, 8, 900, 128, 4), (2, 28, 4, 777, 128, 3),
    (2, 4, 4, 513, 128, 1), (1, 16, 2, 2049, 128, 8), (2, 8, 4, 300, 64, 2), (1, 8, 1, 64, 128, 2),
])
@pytest.mark.parametrize("ragged", [False, True])
def test_decode_matches_oracle(gpu_device, decode_variant, B, Hq, Hkv, S, d, splits, ragged):
    gen = torch.Generator().manual_seed(S * 31 + Hq + splits + ragged)
    q = torch.randn(B, Hq, d, generator=gen).to(torch.bfloat16)
    k = torch.randn(B, Hkv, S + 5, d, generator=gen).to(torch.bfloat16)   # padded cache (S_max > S)
    v = torch.randn(B, Hkv, S + 5, d, generator=gen).to(torch.bfloat16)
    lens = [S if not ragged else max(1, S - 7 * b) for b in range(B)]
    W = max(1, S - 2)
    lw, bias, enable, heads = _bias_inputs(B, Hq, S, W, gen)
    refs = []
    for b in range(B):
        L = lens[b]
        Wb = min(W, L)
        refs.append(hook_ref.biased_attention_ref(q[b:b + 1, :, None], k[b:b + 1, :, :L], v[b:b + 1, :, :L],
                                                  lw[b:b + 1, :Wb], [heads[b]], d ** -0.5)[:, 0])
    ref = torch.cat(refs, 0)
    from cram_amd import ops
    dev = gpu_device
    out = ops.attn_decode(q.to(dev), k.to(dev), v.to(dev), scale=d ** -0.5,
                          seq_lens=torch.tensor(lens, dtype=torch.int32, device=dev),
                          bias=bias.to(dev), enable=enable.to(dev), W=W, num_splits=splits)
    torch.cuda.synchronize()
    _check(out, ref)


@pytest.mark.parametrize("B,Hq,Hkv,S,shared,splits", [
    (5, 32, 8, 900, 37, 1), (3, 32, 8, 900, 64, 2), (4, 28, 4, 777, 40, 1), (3, 28, 4, 777, 96, 3),
    (2, 32, 8, 120, 31, 1), (3, 8, 8, 300, 64, 2)])
def test_decode_shared_rows_bit_identical(gpu_device, decode_variant, B, Hq, Hkv, S, shared, splits):
    """cram_attn_decode_shared (ABI 8): with keys / values [0, shared) equal in every batch row (the decode batch's
    shared opening, copied into each cache row), reading them from row 0 gives the same bits as reading each row's
    copy; ragged lengths, bias, split-S, GQA 4 / 7 (matrix-core body) and MHA (VALU body, which ignores it)."""
    from cram_amd import ops
    dev = gpu_device
    gen = torch.Generator().manual_seed(S + shared + splits)
    q = torch.randn(B, Hq, 128, generator=gen).to(torch.bfloat16).to(dev)
    k = torch.randn(B, Hkv, S + 5, 128, generator=gen).to(torch.bfloat16).to(dev)
    v = torch.randn(B, Hkv, S + 5, 128, generator=gen).to(torch.bfloat16).to(dev)
    k[1:, :, :shared] = k[:1, :, :shared]
    v[1:, :, :shared] = v[:1, :, :shared]
    lens = torch.tensor([max(shared + 1, S - 9 * b) for b in range(B)], dtype=torch.int32, device=dev)
    _, bias, enable, _ = _bias_inputs(B, Hq, S, S - 2, gen)
    kw = dict(scale=128 ** -0.5, seq_lens=lens, bias=bias.to(dev), enable=enable.to(dev), W=S - 2, num_splits=splits)
    a = ops.attn_decode(q, k, v, **kw)
    b = ops.attn_decode(q, k, v, shared_rows=shared, **kw)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    # the indirection is real: poisoning the other rows' copies of whole shared 32-key blocks changes nothing
    if shared >= 32 and Hq // Hkv >= 4 and decode_variant == "auto":
        k[1:, :, :shared // 32 * 32] = 0
        c = ops.attn_decode(q, k, v, shared_rows=shared, **kw)
        assert torch.equal(a, c)


def test_answer_logits(gpu_device):
    gen = torch.Generator().manual_seed(3)
    n, D, V = 37, 4096, 1000
    h = torch.randn(n, D, generator=gen).to(torch.bfloat16)
    w = (torch.randn(V, D, generator=gen) * 0.02).to(torch.bfloat16)
    ids = torch.randint(0, V, (n,), generator=gen, dtype=torch.int32)
    ref = (h.double() * w[ids.long()].double()).sum(-1)
    from cram_amd import ops
    dev = gpu_device
    out = ops.answer_logits(h.to(dev), w.to(dev), ids.to(dev))
    torch.cuda.synchronize()
    assert torch.allclose(out.double().cpu(), ref, atol=1e-3, rtol=1e-4)
    out16 = ops.answer_logits(h.to(dev), w.to(dev), ids.to(dev), round_logits=True)
    assert torch.equal(out16.cpu(), out.cpu().to(torch.bfloat16).float())


def test_rejects_bad_alignment(gpu_device):
    from cram_amd import ops
    dev = gpu_device
    q = torch.randn(1, 2, 4, 100, device=dev).to(torch.bfloat16)   # d = 100 unsupported
    with pytest.raises(RuntimeError):
        ops.attn_prefill(q, q[:, :1], q[:, :1], scale=0.1)


# ----------------------------------------------------------------------------------------------
# fused elementwise kernels vs transformers' op sequences (LlamaRMSNorm, apply_rotary_pos_emb, LlamaMLP)
# ----------------------------------------------------------------------------------------------
def _ulp_diff(a, b):
    """bf16 ulp distance per element."""
    ai = a.view(torch.int16).to(torch.int32)
    bi = b.view(torch.int16).to(torch.int32)
    ai = torch.where(ai < 0, -(ai & 0x7FFF), ai)
    bi = torch.where(bi < 0, -(bi & 0x7FFF), bi)
    return (ai - bi).abs()


@pytest.mark.parametrize("D", [256, 3584, 4096])
@pytest.mark.parametrize("with_residual", [False, True])
def test_rmsnorm_matches_transformers(gpu_device, D, with_residual):
    from cram_amd import ops
    dev = gpu_device
    g = torch.Generator(device=dev).manual_seed(D)
    x = torch.randn(3, 77, D, device=dev, generator=g).to(torch.bfloat16)
    r = torch.randn(3, 77, D, device=dev, generator=g).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(D, device=dev, generator=g)).to(torch.bfloat16)
    h = (r + x) if with_residual else x
    hf = h.float()
    ref = w * (hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5)).to(torch.bfloat16)
    if with_residual:
        h_got, got = ops.rmsnorm(x, w, 1e-5, residual=r)
        assert torch.equal(h_got, h)
    else:
        got = ops.rmsnorm(x, w, 1e-5)
    ud = _ulp_diff(got, ref)
    assert ud.max() <= 1 and (ud == 0).float().mean() > 0.995, (ud.max().item(), (ud == 0).float().mean().item())


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (28, 4), (4, 2)])
def test_rope_bit_exact(gpu_device, Hq, Hkv):
    from cram_amd import ops
    from cram_amd.engine import CrAMEngine, ModelSpec
    dev = gpu_device
    d = 128
    sp = ModelSpec(1, Hq * d, Hq, Hkv, d, 256, 100, 1e-5, False)
    eng = CrAMEngine.random(sp, dev, seed=1)
    B, T = 2, 131
    N = (Hq + 2 * Hkv) * d
    y = torch.randn(B, T, N, device=dev).to(torch.bfloat16)
    cos, sin = eng.rope_tables(T)
    # transformers: q_embed = (q * cos) + (rotate_half(q) * sin), heads unsqueezed
    x = y[..., :(Hq + Hkv) * d].unflatten(-1, (Hq + Hkv, d))
    c, s = cos[None, :, None, :], sin[None, :, None, :]
    rot = torch.cat((-x[..., d // 2:], x[..., :d // 2]), dim=-1)
    ref = (x * c) + (rot * s)
    v_before = y[..., (Hq + Hkv) * d:].clone()
    ops.rope_inplace(y, Hq + Hkv, d, cos, sin, T)
    assert torch.equal(y[..., :(Hq + Hkv) * d].unflatten(-1, (Hq + Hkv, d)), ref)
    assert torch.equal(y[..., (Hq + Hkv) * d:], v_before)
    # per-row positions (decode)
    y2 = torch.randn(5, 1, N, device=dev).to(torch.bfloat16)
    pos = torch.tensor([0, 7, 130, 64, 3], device=dev)
    x2 = y2[:, 0, :(Hq + Hkv) * d].unflatten(-1, (Hq + Hkv, d))
    rot2 = torch.cat((-x2[..., d // 2:], x2[..., :d // 2]), dim=-1)
    ref2 = (x2 * cos[pos][:, None]) + (rot2 * sin[pos][:, None])
    ops.rope_inplace(y2, Hq + Hkv, d, cos, sin, 1, pos=pos)
    assert torch.equal(y2[:, 0, :(Hq + Hkv) * d].unflatten(-1, (Hq + Hkv, d)), ref2)


@pytest.mark.parametrize("Hq,Hkv,dtype", [(32, 8, torch.bfloat16), (28, 4, torch.bfloat16), (4, 2, torch.float16)])
def test_rope_split_equals_inplace_plus_copy(gpu_device, Hq, Hkv, dtype):
    """cram_rope_split (the IE sweep's suffix layers): q rotated in place and k/v written behind a prefix in
    [B, p0 + T] buffers, bit-identical to cram_rope_inplace followed by the copies it replaces; per-row positions
    p0 + t, a padded row buffer, and the prefix rows left untouched."""
    from cram_amd import ops
    from cram_amd.engine import CrAMEngine, ModelSpec
    dev = gpu_device
    d = 128
    sp = ModelSpec(1, Hq * d, Hq, Hkv, d, 256, 100, 1e-5, False)
    eng = CrAMEngine.random(sp, dev, seed=1, dtype=dtype)
    B, T, p0 = 5, 77, 19
    N = (Hq + 2 * Hkv) * d
    cos, sin = eng.rope_tables(p0 + T)
    ybuf = torch.randn(B * T + 64, N, device=dev).to(dtype)          # padded rows beyond B * T
    pos = (torch.arange(T, device=dev) + p0).repeat(B)
    y_ref = ybuf[:B * T].clone()
    ops.rope_inplace(y_ref, Hq + Hkv, d, cos, sin, T, pos=pos)
    y3 = y_ref.view(B, T, N)
    k_ref = y3[..., Hq * d:(Hq + Hkv) * d].unflatten(-1, (Hkv, d))
    v_ref = y3[..., (Hq + Hkv) * d:].unflatten(-1, (Hkv, d))
    k = torch.randn(B, p0 + T, Hkv, d, device=dev).to(dtype)
    v = torch.randn_like(k)
    k_pre, v_pre = k[:, :p0].clone(), v[:, :p0].clone()
    pad_before = ybuf[B * T:].clone()
    ops.rope_split(ybuf[:B * T], Hq, Hkv, d, cos, sin, T, k, v, p0, pos=pos)
    assert torch.equal(ybuf[:B * T, :Hq * d], y_ref[:, :Hq * d])
    assert torch.equal(k[:, p0:], k_ref) and torch.equal(v[:, p0:], v_ref)
    assert torch.equal(k[:, :p0], k_pre) and torch.equal(v[:, :p0], v_pre)
    assert torch.equal(ybuf[B * T:], pad_before)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_rope_split_scatter_into_cache(gpu_device, dtype):
    """The packed decode prefill's form of cram_rope_split: q and k roped in place (keep_k), and the roped k / the v
    of packed row r written to cache row pos[r] of sequence dst_b[r] in the head-major [B, Hkv, S, d] cache, bit-
    identical to rope_inplace followed by the index_put it replaces; untouched cache rows stay as they were."""
    from cram_amd import ops
    from cram_amd.engine import CrAMEngine, ModelSpec
    dev = gpu_device
    Hq, Hkv, d = 32, 8, 128
    sp = ModelSpec(1, Hq * d, Hq, Hkv, d, 256, 100, 1e-5, False)
    eng = CrAMEngine.random(sp, dev, seed=2, dtype=dtype)
    B, S = 6, 200
    lens = [37, 1, 120, 64, 5, 90]
    pos = torch.cat([torch.arange(n) for n in lens]).to(dev)
    bidx = torch.cat([torch.full((n,), b) for b, n in enumerate(lens)]).to(dev)
    total, N = sum(lens), (Hq + 2 * Hkv) * d
    cos, sin = eng.rope_tables(S)
    y = torch.randn(total, N, device=dev).to(dtype)
    y_ref = y.clone()
    ops.rope_inplace(y_ref, Hq + Hkv, d, cos, sin, 1, pos=pos)
    kc = torch.randn(B, Hkv, S, d, device=dev).to(dtype)
    vc = torch.randn_like(kc)
    kc_ref, vc_ref = kc.clone(), vc.clone()
    kc_ref[bidx, :, pos] = y_ref[:, Hq * d:(Hq + Hkv) * d].view(total, Hkv, d)
    vc_ref[bidx, :, pos] = y_ref[:, (Hq + Hkv) * d:].view(total, Hkv, d)
    ops.rope_split(y, Hq, Hkv, d, cos, sin, 1, kc.transpose(1, 2), vc.transpose(1, 2), 0, pos=pos, dst_b=bidx,
                   keep_k=True)
    assert torch.equal(y, y_ref)
    assert torch.equal(kc, kc_ref) and torch.equal(vc, vc_ref)


@pytest.mark.parametrize("F", [512, 14336, 18944])
def test_silu_mul_matches_transformers(gpu_device, F):
    from cram_amd import ops
    dev = gpu_device
    gu = (2 * torch.randn(3, 50, 2 * F, device=dev)).to(torch.bfloat16)
    ref = torch.nn.functional.silu(gu[..., :F]) * gu[..., F:]
    got = ops.silu_mul(gu, F)
    ud = _ulp_diff(got, ref)
    assert ud.max() <= 1 and (ud == 0).float().mean() > 0.995, (ud.max().item(), (ud == 0).float().mean().item())


@pytest.mark.parametrize("lens,Hq,Hkv", [([17, 300, 1, 129], 8, 2), ([900, 77], 32, 8), ([5, 6, 7], 7, 1)])
def test_prefill_varlen_matches_oracle(gpu_device, prefill_variant, lens, Hq, Hkv):
    """Packed sequences (cu_seqlens) in one launch == each sequence through the oracle."""
    from cram_amd import ops
    gen = torch.Generator().manual_seed(sum(lens))
    d = 128
    total = sum(lens)
    N = (Hq + 2 * Hkv) * d
    y = torch.randn(total, N, generator=gen).to(torch.bfloat16)      # packed fused-QKV rows
    q = y[:, :Hq * d].view(total, Hq, d)
    k = y[:, Hq * d:(Hq + Hkv) * d].view(total, Hkv, d)
    v = y[:, (Hq + Hkv) * d:].view(total, Hkv, d)
    W = max(lens)
    lw, bias, enable, heads = _bias_inputs(len(lens), Hq, W, W, gen)
    cu = [0]
    for n in lens:
        cu.append(cu[-1] + n)
    refs = []
    for b, n in enumerate(lens):
        a, e = cu[b], cu[b + 1]
        refs.append(hook_ref.biased_attention_ref(q[a:e].transpose(0, 1)[None], k[a:e].transpose(0, 1)[None],
                                                  v[a:e].transpose(0, 1)[None], lw[b:b + 1, :n], [heads[b]],
                                                  d ** -0.5)[0])
    ref = torch.cat(refs, 0)
    dev = gpu_device
    yd = y.to(dev)
    out = ops.attn_prefill_varlen(yd[:, :Hq * d].view(total, Hq, d), yd[:, Hq * d:(Hq + Hkv) * d].view(total, Hkv, d),
                                  yd[:, (Hq + Hkv) * d:].view(total, Hkv, d),
                                  torch.tensor(cu, dtype=torch.int32, device=dev), max(lens), scale=d ** -0.5,
                                  bias=bias.to(dev), enable=enable.to(dev), W=W)
    torch.cuda.synchronize()
    _check(out, ref)


@pytest.mark.parametrize("prefix,lens,Hq,Hkv", [(37, [300, 17, 129, 1], 32, 8), (16, [900, 77], 8, 2),
                                                (64, [5, 6, 7], 7, 1)])
def test_prefill_varlen_cached_matches_oracle(gpu_device, prefill_variant, prefix, lens, Hq, Hkv):
    """Packed prompt suffixes over a KV cache holding a shared prefix (cram_attn_prefill_varlen_cached, the batched
    decode's prefill with the chat-template opening computed once) == each sequence's suffix rows through the oracle
    over [prefix | suffix] keys, with the bias on absolute key positions."""
    from cram_amd import ops
    gen = torch.Generator().manual_seed(prefix + sum(lens))
    d, B = 128, len(lens)
    S_max = prefix + max(lens) + 8
    bf = torch.bfloat16
    kc = torch.zeros((B, Hkv, S_max, d), dtype=bf)
    vc = torch.zeros_like(kc)
    kc[:, :, :prefix] = torch.randn(Hkv, prefix, d, generator=gen).to(bf)
    vc[:, :, :prefix] = torch.randn(Hkv, prefix, d, generator=gen).to(bf)
    W = prefix + max(lens)
    lw, bias, enable, heads = _bias_inputs(B, Hq, W, W, gen)
    qs, refs, cu = [], [], [0]
    for b, n in enumerate(lens):
        kc[b, :, prefix:prefix + n] = torch.randn(Hkv, n, d, generator=gen).to(bf)
        vc[b, :, prefix:prefix + n] = torch.randn(Hkv, n, d, generator=gen).to(bf)
        q = torch.randn(Hq, n, d, generator=gen).to(bf)
        S = prefix + n
        refs.append(hook_ref.biased_attention_ref(q[None], kc[b:b + 1, :, :S], vc[b:b + 1, :, :S],
                                                  lw[b:b + 1, :min(W, S)], [heads[b]], d ** -0.5)[0])
        qs.append(q.transpose(0, 1))
        cu.append(cu[-1] + n)
    dev = gpu_device
    kd, vd = kc.to(dev), vc.to(dev)
    out = ops.attn_prefill_varlen_cached(torch.cat(qs).contiguous().to(dev), kd.transpose(1, 2), vd.transpose(1, 2),
                                         torch.tensor(cu, dtype=torch.int32, device=dev), max(lens), prefix,
                                         scale=d ** -0.5, bias=bias.to(dev), enable=enable.to(dev), W=W)
    torch.cuda.synchronize()
    _check(out, torch.cat(refs, 0))


def _rows_ref(q, k, v, bias, enable, W, scale, b, h, rows, G):
    """float64 reference for a few query rows of one (batch, head): causal over keys <= row (q_pos0 = 0),
    bias[b, j] added for j < W when the head is enabled (the hook's semantics, re_weighting.py:57-59)."""
    out = []
    kk = k[b, h // G].double()
    vv = v[b, h // G].double()
    for i in rows:
        s = (kk[:i + 1] @ q[b, h, i].double()) * scale
        if bias is not None and enable[b, h]:
            jb = min(i + 1, W)
            s[:jb] += bias[b, :jb].double()
        p = torch.softmax(s, 0)
        out.append(p @ vv[:i + 1])
    return torch.stack(out)


@pytest.mark.parametrize("B,T", [(33, 962), (1, 8300)])
def test_prefill_full_size_properties(gpu_device, prefill_variant, B, T):
    """BASELINE sizes (the IE sweep's 33-variant batch at T' = 962; config 5's 8k prompt), Llama-3 GQA 32/8.
    Size-independent properties, bit-exact: zero bias on every head == no bias; each batch element equals
    its own single-sequence launch; two q-heads of one GQA group with equal queries give equal outputs.
    Sampled rows (first, tile edges, last) of biased heads with -inf and 0.1 spans vs float64 (the usual
    bf16 tolerance)."""
    from cram_amd import ops
    dev = gpu_device
    Hq, Hkv, d = 32, 8, 128
    G = Hq // Hkv
    g = torch.Generator(device=dev).manual_seed(B * 7 + T)
    q = torch.randn(B, T, Hq, d, generator=g, device=dev).to(torch.bfloat16).transpose(1, 2)
    with torch.no_grad():
        q[:, 5] = q[:, 4]                                           # heads 4, 5: same kv head (G = 4)
    k = torch.randn(B, Hkv, T, d, generator=g, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Hkv, T, d, generator=g, device=dev).to(torch.bfloat16)
    scale = d ** -0.5
    plain = ops.attn_prefill(q, k, v, scale=scale)
    zero = ops.attn_prefill(q, k, v, scale=scale, bias=torch.zeros(B, T, device=dev),
                            enable=torch.ones(B, Hq, dtype=torch.uint8, device=dev), W=T)
    assert torch.equal(plain, zero)
    assert torch.equal(plain[:, :, 4], plain[:, :, 5])
    for b in sorted({0, B // 2, B - 1}):
        one = ops.attn_prefill(q[b:b + 1], k[b:b + 1], v[b:b + 1], scale=scale)
        assert torch.equal(one[0], plain[b])
    W = T - 5
    w = torch.ones(B, W, dtype=torch.float16)
    w[:, 30:200] = 0.0                                              # -inf span (score 0)
    w[:, 400:700] = 0.1                                             # log 0.1 span
    bias = hook_ref.log_weight(w).to(torch.bfloat16).float()
    enable = torch.zeros(B, Hq, dtype=torch.uint8)
    enable[:, ::3] = 1
    out = ops.attn_prefill(q, k, v, scale=scale, bias=bias.to(dev), enable=enable.to(dev), W=W)
    torch.cuda.synchronize()
    rows = [0, 1, 63, 64, 250, T // 2, T - 1]
    qc, kc, vc, oc = q.cpu(), k.cpu(), v.cpu(), out.cpu()
    for b in sorted({0, B - 1}):
        for h in (0, 1, 3, Hq - 1):
            ref = _rows_ref(qc, kc, vc, bias, enable, W, scale, b, h, rows, G)
            _check(oc[b, rows, h], ref)


def test_varlen_full_size_equals_dense(gpu_device, prefill_variant):
    """Config 2's packed prefill shape (64 prompts of 700-1100 tokens): every packed sequence equals its own
    dense single-sequence launch bit for bit (same tiles, same arithmetic)."""
    from cram_amd import ops
    dev = gpu_device
    Hq, Hkv, d = 32, 8, 128
    g = torch.Generator(device=dev).manual_seed(11)
    lens = torch.randint(700, 1101, (64,), generator=torch.Generator().manual_seed(3)).tolist()
    total = sum(lens)
    qkv = torch.randn(total, (Hq + 2 * Hkv) * d, generator=g, device=dev).to(torch.bfloat16)
    q = qkv[:, :Hq * d].view(total, Hq, d)
    k = qkv[:, Hq * d:(Hq + Hkv) * d].view(total, Hkv, d)
    v = qkv[:, (Hq + Hkv) * d:].view(total, Hkv, d)
    cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device=dev)
    out = ops.attn_prefill_varlen(q, k, v, cu, max(lens), scale=d ** -0.5)
    for i in (0, 17, 63):
        a, n = int(cu[i]), lens[i]
        one = ops.attn_prefill(q[a:a + n].transpose(0, 1)[None], k[a:a + n].transpose(0, 1)[None],
                               v[a:a + n].transpose(0, 1)[None], scale=d ** -0.5)
        assert torch.equal(one[0], out[a:a + n])


# every decode grid the bench times: (name, rows, Hq, Hkv, S_max, prompt-length range); split count by the engine's rule
DECODE_GRIDS = [
    ("config2_b256", 256, 32, 8, 1152, (700, 1101)),
    ("config2_b512", 512, 32, 8, 1216, (700, 1101)),      # bench --decode-batch 512 (NQ-1000 = 2 x 500 rows)
    ("config4_b500", 500, 28, 4, 1216, (700, 1101)),      # Qwen2-7B heads, TriviaQA-1000 = 2 x 500 rows
    ("config5_b143", 143, 32, 8, 8448, (8000, 8349)),     # 20 docs, the KV budget's 143 rows of ~8.3k tokens
    ("config5_b16", 16, 32, 8, 8448, (8000, 8349)),       # the round-3 config-5 batch (split-S)
]


@pytest.mark.parametrize("grid", DECODE_GRIDS, ids=[g[0] for g in DECODE_GRIDS])
def test_decode_full_size_sampled(gpu_device, grid):
    """The decode steps of the bench's grids (rows, heads, cached keys, the engine's split-S count; top-half heads
    biased with a -inf and a 0.1 span) on sampled rows vs float64, and each sampled row bit-identical to a launch of
    that row alone (same split count): rows never interact."""
    from cram_amd import ops
    from cram_amd.engine import decode_attn_splits
    _, B, Hq, Hkv, S_max, (lo, hi) = grid
    dev = gpu_device
    d, G = 128, Hq // Hkv
    g = torch.Generator(device=dev).manual_seed(5)
    q = torch.randn(B, Hq, d, generator=g, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Hkv, S_max, d, generator=g, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Hkv, S_max, d, generator=g, device=dev).to(torch.bfloat16)
    lens = torch.randint(lo, hi, (B,), generator=torch.Generator().manual_seed(9))
    W = lo - 10
    w = torch.ones(B, W, dtype=torch.float16)
    w[:, 20:150] = 0.0
    w[:, 300:500] = 0.1
    bias = hook_ref.log_weight(w).to(torch.bfloat16).float()
    enable = torch.zeros(B, Hq, dtype=torch.uint8)
    enable[:, :Hq // 2] = 1
    splits = decode_attn_splits(B, Hkv, S_max)
    ws = (torch.empty(ops.decode_workspace_bytes(B, Hq, d, splits), dtype=torch.uint8, device=dev)
          if splits > 1 else None)
    lens_d, bias_d, en_d = lens.to(torch.int32).to(dev), bias.to(dev), enable.to(dev)
    out = ops.attn_decode(q, k, v, scale=d ** -0.5, seq_lens=lens_d, bias=bias_d, enable=en_d, W=W,
                          num_splits=splits, workspace=ws).cpu()
    qc, kc, vc = q.cpu(), k.cpu(), v.cpu()
    rows = sorted({0, B // 2 - 1, B - 1})
    for b in rows:
        L = int(lens[b])
        for h in sorted({0, G - 1, Hq // 2 - 1, Hq // 2, Hq - 1}):
            kk, vv = kc[b, h // G, :L].double(), vc[b, h // G, :L].double()
            s = (kk @ qc[b, h].double()) * d ** -0.5
            if enable[b, h]:
                s[:W] += bias[b].double()
            ref = torch.softmax(s, 0) @ vv
            _check(out[b, h][None], ref[None])
        ws1 = (torch.empty(ops.decode_workspace_bytes(1, Hq, d, splits), dtype=torch.uint8, device=dev)
               if splits > 1 else None)
        one = ops.attn_decode(q[b:b + 1], k[b:b + 1], v[b:b + 1], scale=d ** -0.5, seq_lens=lens_d[b:b + 1],
                              bias=bias_d[b:b + 1], enable=en_d[b:b + 1], W=W, num_splits=splits, workspace=ws1).cpu()
        assert torch.equal(one[0], out[b]), f"row {b} differs from its own launch"


def test_plain_c_host_runs(gpu_device):
    """The C-ABI driven from plain C (examples/abi_demo.c): biased prefill vs a double CPU loop + error path."""
    import os
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-C", os.path.join(repo, "examples"), "-s"], check=True)
    r = subprocess.run([os.path.join(repo, "examples", "abi_demo")], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "max|err|" in r.stdout
