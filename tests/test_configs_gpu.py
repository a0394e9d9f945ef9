"""Kernel parity at the shapes of BASELINE configs 1 and 5 that no other GPU test runs.

* Config 1 — GPT-2-small: 12 MHA heads (Hq = Hkv = 12), head_dim 64, NQ prompts of T ~ 890 tokens, every head
  re-weighted (layers_to_be_modified = {} -> all heads, re_weighting.py:32-33).  Prefill at T = 890 and decode
  at S = 890 / 1024 with the split count the cram_hip attention interface picks (cram_amd/attention.py
  _num_splits), against the float64 oracle over the hook's dense mask (re_weighting.py:36-61).
* Config 5 — Llama-3-8B long context: 16 prompts of ~8.3k tokens, 20 retrieved-doc spans (one -inf span of
  score 0, several log 0.1 spans), GQA 32/8, decode at the split count DecodeSession picks for that batch
  (cram_amd/engine.py: ceil(512 / (B * Hkv)) capped by S_max / 256 -> 4), for every decode body U = 4 / 1 / 2.
  Every (row, head) is checked against float64 (one query per head: cheap on the host).
Tolerance: the bf16 bar of tests/test_kernels_gpu.py (|err| <= 2e-2 + 2e-2 |ref|, mean <= 2e-3).
"""
import math

import pytest
import torch

from oracle import hook_ref

pytestmark = pytest.mark.gpu

ATOL, RTOL, MEAN_TOL = 2e-2, 2e-2, 2e-3


def _check(out, ref):
    out = out.double().cpu()
    assert torch.isfinite(out).all()
    err = (out - ref).abs()
    bad = err > ATOL + RTOL * ref.abs()
    assert not bad.any(), f"max err {err.max().item():.3e} at {bad.nonzero()[0].tolist()}"
    assert err.mean().item() < MEAN_TOL, f"mean err {err.mean().item():.3e}"


def _nq_like_weights(B, W, n_spans, gen, fake_score=0.1, with_zero=True):
    """fp16 weights [B, W]: n_spans contiguous passage spans after a 30-token template head; one span per row
    carries fake_score, one (if with_zero) score 0 -> -inf, the rest 1.0 (bias 0)."""
    w = torch.ones((B, W), dtype=torch.float16)
    edges = torch.linspace(30, W - 20, n_spans + 1).long().tolist()
    for b in range(B):
        perm = torch.randperm(n_spans, generator=gen).tolist()
        w[b, edges[perm[0]]:edges[perm[0] + 1]] = fake_score
        if with_zero:
            w[b, edges[perm[1]]:edges[perm[1] + 1]] = 0.0
            w[b, edges[perm[2]]:edges[perm[2] + 1]] = fake_score
    return w


def test_gpt2_small_prefill_all_heads(gpu_device):
    """Config 1 prefill: B = 1, 12 x 12 MHA heads, d = 64, T = 890, all heads re-weighted."""
    from cram_amd import ops
    dev = gpu_device
    gen = torch.Generator().manual_seed(890)
    B, H, T, d = 1, 12, 890, 64
    q = torch.randn(B, T, H, d, generator=gen).to(torch.bfloat16).transpose(1, 2)   # transformers' view
    k = torch.randn(B, H, T, d, generator=gen).to(torch.bfloat16)
    v = torch.randn(B, H, T, d, generator=gen).to(torch.bfloat16)
    w = _nq_like_weights(B, T, 5, gen)
    lw = hook_ref.log_weight(w)
    heads = [list(range(H))]
    bias = lw.to(torch.bfloat16).float()
    enable = torch.ones((B, H), dtype=torch.uint8)
    ref = hook_ref.biased_attention_ref(q, k, v, lw, heads, 1.0 / math.sqrt(d))
    out = ops.attn_prefill(q.to(dev), k.to(dev), v.to(dev), scale=1.0 / math.sqrt(d), bias=bias.to(dev),
                           enable=enable.to(dev), W=T)
    torch.cuda.synchronize()
    _check(out, ref)
    # ideal-score prompts of config 1 (only a 0.1 span): same bar
    w1 = _nq_like_weights(B, T, 5, gen, with_zero=False)
    lw1 = hook_ref.log_weight(w1)
    ref1 = hook_ref.biased_attention_ref(q, k, v, lw1, heads, 1.0 / math.sqrt(d))
    out1 = ops.attn_prefill(q.to(dev), k.to(dev), v.to(dev), scale=1.0 / math.sqrt(d),
                            bias=lw1.to(torch.bfloat16).float().to(dev), enable=enable.to(dev), W=T)
    torch.cuda.synchronize()
    _check(out1, ref1)


@pytest.mark.parametrize("S", [890, 1024])
def test_gpt2_small_decode_all_heads(gpu_device, decode_variant, S):
    """Config 1 decode: one new token over S cached keys (prompt W = 880 tokens + generated keys beyond W, which
    the hook leaves unbiased), 12 MHA heads, d = 64, split count of the attention interface."""
    from cram_amd import ops
    from cram_amd.attention import _num_splits
    dev = gpu_device
    gen = torch.Generator().manual_seed(S)
    B, H, d, W = 1, 12, 64, 880
    q = torch.randn(B, H, d, generator=gen).to(torch.bfloat16)
    k = torch.randn(B, H, S, d, generator=gen).to(torch.bfloat16)
    v = torch.randn(B, H, S, d, generator=gen).to(torch.bfloat16)
    w = _nq_like_weights(B, W, 5, gen)
    lw = hook_ref.log_weight(w)
    ref = hook_ref.biased_attention_ref(q[:, :, None], k, v, lw, [list(range(H))], d ** -0.5)[:, 0]
    splits = _num_splits(B, H, S)
    assert splits == S // 256                                          # 3 / 4: the split path is exercised
    out = ops.attn_decode(q.to(dev), k.to(dev), v.to(dev), scale=d ** -0.5, bias=lw.to(torch.bfloat16).float().to(dev),
                          enable=torch.ones((B, H), dtype=torch.uint8, device=dev), W=W, num_splits=splits)
    torch.cuda.synchronize()
    _check(out, ref)


@pytest.mark.parametrize("B", [16, 143])
def test_config5_decode_long_context(gpu_device, decode_variant, B):
    """Config 5 decode step: B sequences of 8,150-8,400 cached keys (ragged), GQA 32/8, 20 passage spans per prompt
    (a -inf span, log-0.1 spans, 1.0 elsewhere), top-half heads re-weighted, the engine's split count: B = 143 is the
    bench's batch (the rows the KV budget holds: 0.55 x 288 GB / 1.1 GB per row; 2 splits since round 4), B = 16
    the round-3 batch (4 splits).  Every row vs float64 at B = 16, 8 sampled rows at B = 143."""
    from cram_amd import ops
    from cram_amd.engine import decode_attn_splits
    dev = gpu_device
    Hq, Hkv, d = 32, 8, 128
    lens = torch.randint(8150, 8401, (B,), generator=torch.Generator().manual_seed(5)).tolist()
    S_max = (max(lens) + 100 + 63) // 64 * 64                          # DecodeSession: prompt + 100 new, 64-aligned
    splits = decode_attn_splits(B, Hkv, S_max)
    assert splits == {16: 4, 143: 2}[B]
    g = torch.Generator(device=dev).manual_seed(8300)
    q = torch.randn(B, Hq, d, generator=g, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Hkv, S_max, d, generator=g, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Hkv, S_max, d, generator=g, device=dev).to(torch.bfloat16)
    W = min(lens) - 40                                                 # generated keys (>= W) stay unbiased
    w = _nq_like_weights(B, W, 20, torch.Generator().manual_seed(20))
    bias = hook_ref.log_weight(w).to(torch.bfloat16).float()
    assert (bias == -math.inf).any() and (bias == -2.296875).any()
    enable = torch.zeros((B, Hq), dtype=torch.uint8)
    enable[:, ::2] = 1
    ws = (torch.empty(ops.decode_workspace_bytes(B, Hq, d, splits), dtype=torch.uint8, device=dev)
          if splits > 1 else None)
    out = ops.attn_decode(q, k, v, scale=d ** -0.5, seq_lens=torch.tensor(lens, dtype=torch.int32, device=dev),
                          bias=bias.to(dev), enable=enable.to(dev), W=W, num_splits=splits, workspace=ws).cpu()
    rows = list(range(B)) if B <= 16 else sorted({0, 1, 37, 70, 71, 100, B - 2, B - 1})
    qc = q.cpu().double()
    G = Hq // Hkv
    ref = torch.empty((len(rows), Hq, d), dtype=torch.float64)
    for i, b in enumerate(rows):
        L = lens[b]
        kb, vb = k[b, :, :L].cpu().double(), v[b, :, :L].cpu().double()
        for h in range(Hq):
            s = (kb[h // G] @ qc[b, h]) * d ** -0.5
            if enable[b, h]:
                s[:W] += bias[b].double()
            ref[i, h] = torch.softmax(s, 0) @ vb[h // G]
    _check(out[rows], ref)
    # size-independent property: zero bias on every head is bit-identical to no bias
    z = ops.attn_decode(q, k, v, scale=d ** -0.5, seq_lens=torch.tensor(lens, dtype=torch.int32, device=dev),
                        bias=torch.zeros_like(bias).to(dev), enable=torch.ones_like(enable).to(dev), W=W,
                        num_splits=splits, workspace=ws)
    n = ops.attn_decode(q, k, v, scale=d ** -0.5, seq_lens=torch.tensor(lens, dtype=torch.int32, device=dev),
                        num_splits=splits, workspace=ws)
    assert torch.equal(z, n)
