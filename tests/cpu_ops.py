"""Test-only CPU stand-ins for cram_amd.ops (host-logic tests without a GPU).

They let the CPU suite exercise the engine / sweep / transformers-registration
plumbing; the GPU suite runs the same code on the HIP kernels.  Math: fp32
softmax attention with the same bias semantics, result rounded to bf16 like the
kernels' output.
"""
import contextlib
import math

import torch


def attn_prefill(q, k, v, *, scale, q_pos0=None, bias=None, enable=None, W=0, out=None):
    B, Hq, Tq, d = q.shape
    _, Hkv, S, _ = k.shape
    if q_pos0 is None:
        q_pos0 = S - Tq
    G = Hq // Hkv
    kk = k.float().repeat_interleave(G, 1)
    vv = v.float().repeat_interleave(G, 1)
    s = torch.matmul(q.float(), kk.transpose(-1, -2)) * scale
    qi = torch.arange(Tq)[:, None] + q_pos0
    kj = torch.arange(S)[None, :]
    s = s.masked_fill(kj > qi, float("-inf"))
    if bias is not None and enable is not None and W > 0:
        add = torch.zeros((B, S))
        Wc = min(W, S)
        add[:, :Wc] = bias[:, :Wc].float().cpu()
        en = enable.cpu().bool()[:, :, None, None]
        add = torch.where(en, add[:, None, None, :], torch.zeros(()))
        s = s + add
    p = torch.softmax(s, -1)
    o = torch.matmul(p, vv).to(q.dtype).transpose(1, 2).contiguous()
    if out is not None:
        out.copy_(o)
        return out
    return o


def attn_decode(q, k, v, *, scale, seq_lens=None, bias=None, enable=None, W=0, num_splits=1, workspace=None,
                out=None, shared_rows=0):
    B, Hq, d = q.shape
    outs = []
    for b in range(B):
        L = int(seq_lens[b]) if seq_lens is not None else k.shape[2]
        o = attn_prefill(q[b:b + 1, :, None], k[b:b + 1, :, :L], v[b:b + 1, :, :L], scale=scale, q_pos0=L - 1,
                         bias=None if bias is None else bias[b:b + 1], enable=None if enable is None else enable[b:b + 1],
                         W=min(W, L))
        outs.append(o[:, 0])
    o = torch.cat(outs, 0)
    if out is not None:
        out.copy_(o)
        return out
    return o


def attn_prefill_varlen(q, k, v, cu_seqlens, max_len, *, scale, bias=None, enable=None, W=0, out=None):
    cu = cu_seqlens.tolist()
    res = torch.empty(q.shape, dtype=q.dtype)
    for b in range(len(cu) - 1):
        a, e = cu[b], cu[b + 1]
        o = attn_prefill(q[a:e].transpose(0, 1)[None], k[a:e].transpose(0, 1)[None], v[a:e].transpose(0, 1)[None],
                         scale=scale, bias=None if bias is None else bias[b:b + 1],
                         enable=None if enable is None else enable[b:b + 1], W=W)
        res[a:e] = o[0]
    if out is not None:
        out.copy_(res)
        return out
    return res


def attn_prefill_varlen_cached(q, k, v, cu_seqlens, max_len, prefix, *, scale, bias=None, enable=None, W=0,
                               out=None):
    cu = cu_seqlens.tolist()
    res = torch.empty(q.shape, dtype=q.dtype)
    for b in range(len(cu) - 1):
        a, e = cu[b], cu[b + 1]
        S = prefix + e - a
        o = attn_prefill(q[a:e].transpose(0, 1)[None], k[b:b + 1, :S].transpose(1, 2), v[b:b + 1, :S].transpose(1, 2),
                         scale=scale, q_pos0=prefix, bias=None if bias is None else bias[b:b + 1],
                         enable=None if enable is None else enable[b:b + 1], W=W)
        res[a:e] = o[0]
    if out is not None:
        out.copy_(res)
        return out
    return res


def answer_logits(hidden, w_lm, ids, *, round_logits=False, out=None):
    r = (hidden.float() * w_lm[ids.long()].float()).sum(-1)
    if round_logits:
        r = r.to(hidden.dtype).float()
    return r


def decode_workspace_bytes(B, Hq, d, num_splits):
    return 0


def rmsnorm(x, w, eps, residual=None, h_out=None, out=None):
    h = x if residual is None else (residual + x)
    hf = h.float()
    y = w * (hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype)
    return (h, y) if residual is not None else y


def rope_inplace(qkv, heads, head_dim, cos, sin, T, pos=None):
    shp = qkv.shape
    y = qkv.reshape(-1, shp[-1])
    rows = y.shape[0]
    p = pos.reshape(-1) if pos is not None else torch.arange(rows) % T
    c, s_ = cos[p][:, None, :], sin[p][:, None, :]
    x = y[:, :heads * head_dim].view(rows, heads, head_dim)
    h = head_dim // 2
    rot = torch.cat((-x[..., h:], x[..., :h]), dim=-1)
    y[:, :heads * head_dim] = ((x * c) + (rot * s_)).reshape(rows, -1)
    return qkv


def rope_split(qkv, hq, hkv, head_dim, cos, sin, T, kout, vout, row0, pos=None, dst_b=None, keep_k=False):
    y = qkv.reshape(-1, qkv.shape[-1])
    q_size, kv = hq * head_dim, hkv * head_dim
    k_raw = y[:, q_size:q_size + kv].clone()
    rope_inplace(y, hq + hkv, head_dim, cos, sin, T, pos)
    k_rot = y[:, q_size:q_size + kv].reshape(-1, hkv, head_dim)
    v = y[:, q_size + kv:q_size + 2 * kv].reshape(-1, hkv, head_dim)
    if dst_b is None:
        B = y.shape[0] // T
        kout[:, row0:row0 + T] = k_rot.reshape(B, T, hkv, head_dim)
        vout[:, row0:row0 + T] = v.reshape(B, T, hkv, head_dim)
    else:
        kout[dst_b, row0 + pos] = k_rot
        vout[dst_b, row0 + pos] = v
    if not keep_k:
        y[:, q_size:q_size + kv] = k_raw


def silu_mul(gu, F, out=None):
    return torch.nn.functional.silu(gu[..., :F]) * gu[..., F:]


def gemm_splitk_workspace_bytes(M, N, splits):
    return int(splits) * int(M) * int(N) * 4


def gemm_splitk(x, w, splits, epilogue=0, bias=None, workspace=None, out=None, name=None):
    """cram_gemm_splitk on the CPU: fp32 product (+ bias) rounded once; epilogue 2 = SiLU-mul on [gate; up]."""
    acc = x.float() @ w.float().t()
    if epilogue == 2:
        F = w.shape[0] // 2
        g = acc[..., :F].to(x.dtype).float()
        r = (torch.nn.functional.silu(g).to(x.dtype).float() * acc[..., F:].to(x.dtype).float()).to(x.dtype)
    else:
        r = (acc + bias.float() if bias is not None else acc).to(x.dtype)
    if out is not None:
        out.copy_(r)
        return out
    return r


@contextlib.contextmanager
def patched_ops():
    """Route cram_amd.ops through the CPU stand-ins for the duration of a CPU test."""
    from cram_amd import ops
    names = ("attn_prefill", "attn_prefill_varlen", "attn_prefill_varlen_cached", "attn_decode", "answer_logits", "decode_workspace_bytes",
             "rmsnorm", "rope_inplace", "rope_split", "silu_mul", "gemm_splitk", "gemm_splitk_workspace_bytes")
    saved = {n: getattr(ops, n) for n in names}
    g = globals()
    for n in names:
        setattr(ops, n, g[n])
    try:
        yield
    finally:
        for n, f in saved.items():
            setattr(ops, n, f)


del math
