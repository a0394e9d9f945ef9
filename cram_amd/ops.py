"""torch-tensor front end of the C-ABI (device memory + stream plumbing only).

Every function here validates shapes/dtypes on the host, then enqueues the HIP
kernel on torch's current stream through ``include/cram_attn.h``.  Nothing
falls back to PyTorch math: a missing library or a rejected shape raises.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib, gemm_tune


class KernelTimer:
    """Optional live timing of kernel launches with HIP events on the launch stream (bench roofline).

    When enabled, every launch of a named kernel is bracketed by two events on
    torch's current stream (the stream the kernel is enqueued on) and its
    algorithmic flops / bytes are recorded; `summary()` syncs and reduces.
    """

    def __init__(self):
        self.enabled = False
        self.rec = {}

    def record(self, name, flops, nbytes, dev):
        if not self.enabled:
            return None
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record(torch.cuda.current_stream(dev))
        self.rec.setdefault(name, []).append((s, e, float(flops), float(nbytes), dev))
        return e

    def summary(self):
        out = {}
        for name, rows in self.rec.items():
            torch.cuda.synchronize()
            ms = [s.elapsed_time(e) for s, e, *_ in rows]
            out[name] = {"launches": len(rows), "total_ms": sum(ms), "avg_ms": sum(ms) / len(ms),
                         "flops": sum(r[2] for r in rows), "bytes": sum(r[3] for r in rows)}
        return out

    def reset(self):
        self.rec = {}


TIMER = KernelTimer()


def prefill_kernel_name(dtype: str, Hq: int, Hkv: int, Tq: int, d: int = 128) -> str:
    """The kernel cram_prefill launches for such a call under the current knob (the selection rule of launch_prefill,
    csrc/cram_attn.hip; labels the bench line's roofline kernel)."""
    kv = _lib.get_knob(_lib.KNOB_PREFILL_VARIANT)
    G = Hq // Hkv
    if d == 128 and dtype == "bf16" and G % 4 == 0:
        if kv == 4 or (kv == -1 and Tq >= 256):
            return "prefill_x32_kernel"
    if d == 128 and G % 7 == 0 and (kv == 7 or (kv == -1 and Tq <= 2048)):
        return "prefill_kernel<7 waves>"
    return {3: "prefill_kernel<32-key tiles>", 8: "prefill_kernel<8 waves>"}.get(kv, "prefill_kernel")


def prefill_work(B, Hq, Hkv, Tq, S, d, q_pos0):
    """Algorithmic flops and HBM bytes of one causal prefill launch."""
    visible = Tq * q_pos0 + Tq * (Tq + 1) / 2.0            # sum over queries of visible keys
    flops = 4.0 * d * Hq * B * visible
    nbytes = 2.0 * (2 * B * Hq * Tq * d + 2 * B * Hkv * S * d) + 4.0 * B * S
    return flops, nbytes


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """F.linear (hipBLASLt / rocBLAS GEMM), timed as "gemm" when the bench's KernelTimer is on.  A row count pinned
    for decode steps only runs the default pick inside the sweep / prefill (gemm_tune.shadowed)."""
    M = x.numel() // x.shape[-1]
    if gemm_tune.shadowed(M):
        with gemm_tune.unpinned():
            return _linear(x, w, b, M)
    return _linear(x, w, b, M)


def _linear(x, w, b, M):
    if not TIMER.enabled:
        return torch.nn.functional.linear(x, w, b)
    N, K = w.shape
    ev = TIMER.record("gemm", 2.0 * M * N * K, 2.0 * (M * K + N * K + M * N), x.device)
    y = torch.nn.functional.linear(x, w, b)
    ev.record(torch.cuda.current_stream(x.device))
    return y


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


# element types of the kernels (include/cram_attn.h CRAM_DTYPE_*): the model dtype the reference loads with
# dtype="auto" (bf16 for Llama-3 / Qwen2, fp16 for Llama-2 checkpoints)
DTYPES = {torch.bfloat16: 0, torch.float16: 1}


def _dt(t: torch.Tensor) -> int:
    try:
        return DTYPES[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported element type {t.dtype}: the kernels take bfloat16 or float16") from None


def _check16(name: str, t: torch.Tensor, ndim: int, like: Optional[torch.Tensor] = None) -> None:
    _dt(t)
    if like is not None and t.dtype != like.dtype:
        raise TypeError(f"{name} is {t.dtype} but the other operands are {like.dtype}")
    if t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D, got shape {tuple(t.shape)}")
    if t.stride(-1) != 1:
        raise ValueError(f"{name} must have a contiguous last dimension")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")


def _bias_args(bias, enable, B, Hq, W):
    if bias is None or enable is None:
        return None, 0, None, 0, 0
    if bias.dtype != torch.float32 or bias.dim() != 2 or bias.shape[0] != B or bias.stride(1) != 1:
        raise ValueError("bias must be float32 [B, S] with a contiguous last dim")
    if enable.dtype != torch.uint8 or enable.dim() != 2 or enable.shape != (B, Hq) or enable.stride(1) != 1:
        raise ValueError("enable must be uint8 [B, Hq]")
    if not 0 <= W <= bias.shape[1]:
        raise ValueError(f"W={W} outside the bias row length {bias.shape[1]}")
    return bias.data_ptr(), bias.stride(0), enable.data_ptr(), enable.stride(0), int(W)


def attn_prefill(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, *, scale: float, q_pos0: Optional[int] = None,
                 bias: Optional[torch.Tensor] = None, enable: Optional[torch.Tensor] = None, W: int = 0,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Causal credibility-biased attention for q_len >= 1.

    q [B, Hq, Tq, d], k/v [B, Hkv, S, d] (any strides, last dim contiguous).
    Returns ``out`` [B, Tq, Hq, d] (the layout transformers' attention
    interface returns); query i sits at position ``q_pos0 + i`` (default S - Tq).
    """
    _check16("q", q, 4)
    _check16("k", k, 4, q)
    _check16("v", v, 4, q)
    B, Hq, Tq, d = q.shape
    _, Hkv, S, _ = k.shape
    if k.shape[0] != B or v.shape != k.shape or k.shape[3] != d:
        raise ValueError(f"shape mismatch q{tuple(q.shape)} k{tuple(k.shape)} v{tuple(v.shape)}")
    if q_pos0 is None:
        q_pos0 = S - Tq
    if out is None:
        out = torch.empty((B, Tq, Hq, d), dtype=q.dtype, device=q.device)
    elif out.shape != (B, Tq, Hq, d) or out.dtype != q.dtype or out.stride(-1) != 1:
        raise ValueError("out must be [B, Tq, Hq, d] of q's dtype with a contiguous last dim")
    bp, bsb, ep, esb, W = _bias_args(bias, enable, B, Hq, W)
    lib = _lib.load()
    ev = TIMER.record("cram_prefill", *prefill_work(B, Hq, Hkv, Tq, S, d, q_pos0), q.device) if TIMER.enabled else None
    code = lib.cram_attn_prefill(
        q.data_ptr(), q.stride(0), q.stride(1), q.stride(2),
        k.data_ptr(), k.stride(0), k.stride(1), k.stride(2),
        v.data_ptr(), v.stride(0), v.stride(1), v.stride(2),
        out.data_ptr(), out.stride(0), out.stride(2), out.stride(1),
        B, Hq, Hkv, Tq, S, d, int(q_pos0), float(scale),
        bp, bsb, ep, esb, W, _dt(q), _stream(q.device))
    _lib.check(code, "cram_attn_prefill")
    if ev is not None:
        ev.record(torch.cuda.current_stream(q.device))
    return out


def attn_prefill_varlen(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cu_seqlens: torch.Tensor, max_len: int, *,
                        scale: float, bias: Optional[torch.Tensor] = None, enable: Optional[torch.Tensor] = None,
                        W: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Packed causal attention: q [total, Hq, d], k/v [total, Hkv, d] (token-major, any token stride),
    sequence b = tokens [cu[b], cu[b+1]).  Returns out [total, Hq, d]."""
    _check16("q", q, 3)
    _check16("k", k, 3, q)
    _check16("v", v, 3, q)
    total, Hq, d = q.shape
    Hkv = k.shape[1]
    B = cu_seqlens.numel() - 1
    if cu_seqlens.dtype != torch.int32 or not cu_seqlens.is_cuda or B <= 0:
        raise ValueError("cu_seqlens must be a device int32 [B+1] tensor")
    if out is None:
        out = torch.empty((total, Hq, d), dtype=q.dtype, device=q.device)
    bp, bsb, ep, esb, W = _bias_args(bias, enable, B, Hq, W)
    flops, nbytes = prefill_work(1, Hq, Hkv, max_len, max_len, d, 0)
    ev = TIMER.record("cram_prefill_varlen", flops * B, nbytes * B, q.device) if TIMER.enabled else None
    code = _lib.load().cram_attn_prefill_varlen(
        q.data_ptr(), q.stride(1), q.stride(0), k.data_ptr(), k.stride(1), k.stride(0),
        v.data_ptr(), v.stride(1), v.stride(0), out.data_ptr(), out.stride(1), out.stride(0),
        cu_seqlens.data_ptr(), B, int(max_len), Hq, Hkv, d, float(scale), bp, bsb, ep, esb, W, _dt(q),
        _stream(q.device))
    _lib.check(code, "cram_attn_prefill_varlen")
    if ev is not None:
        ev.record(torch.cuda.current_stream(q.device))
    return out


def attn_prefill_varlen_cached(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cu_seqlens: torch.Tensor,
                               max_len: int, prefix: int, *, scale: float, bias: Optional[torch.Tensor] = None,
                               enable: Optional[torch.Tensor] = None, W: int = 0,
                               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Packed prompt suffixes over cached keys: q [total, Hq, d] (sequence b = tokens [cu[b], cu[b+1]), at positions
    prefix + i), k/v [B, S, Hkv, d] views of the KV cache (token-major, any strides) whose rows 0 .. prefix + len_b - 1
    hold the shared prefix and sequence b's own keys.  Returns out [total, Hq, d]."""
    _check16("q", q, 3)
    _check16("k", k, 4, q)
    _check16("v", v, 4, q)
    total, Hq, d = q.shape
    B, S, Hkv, _ = k.shape
    if v.shape != k.shape or k.shape[3] != d:
        raise ValueError(f"shape mismatch q{tuple(q.shape)} k{tuple(k.shape)} v{tuple(v.shape)}")
    if cu_seqlens.dtype != torch.int32 or not cu_seqlens.is_cuda or cu_seqlens.numel() != B + 1:
        raise ValueError("cu_seqlens must be a device int32 [B+1] tensor (one entry per cache row + 1)")
    if prefix < 0 or prefix + max_len > S:
        raise ValueError(f"prefix {prefix} + max_len {max_len} exceeds the cache's {S} rows")
    if out is None:
        out = torch.empty((total, Hq, d), dtype=q.dtype, device=q.device)
    bp, bsb, ep, esb, W = _bias_args(bias, enable, B, Hq, W)
    flops, nbytes = prefill_work(1, Hq, Hkv, max_len, prefix + max_len, d, prefix)
    ev = TIMER.record("cram_prefill_varlen", flops * B, nbytes * B, q.device) if TIMER.enabled else None
    code = _lib.load().cram_attn_prefill_varlen_cached(
        q.data_ptr(), q.stride(1), q.stride(0), k.data_ptr(), k.stride(0), k.stride(2), k.stride(1),
        v.data_ptr(), v.stride(0), v.stride(2), v.stride(1), out.data_ptr(), out.stride(1), out.stride(0),
        cu_seqlens.data_ptr(), B, int(max_len), int(prefix), Hq, Hkv, d, float(scale), bp, bsb, ep, esb, W, _dt(q),
        _stream(q.device))
    _lib.check(code, "cram_attn_prefill_varlen_cached")
    if ev is not None:
        ev.record(torch.cuda.current_stream(q.device))
    return out


def decode_workspace_bytes(B: int, Hq: int, d: int, num_splits: int) -> int:
    return int(_lib.load().cram_attn_decode_workspace_size(B, Hq, d, num_splits))


def attn_decode(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, *, scale: float,
                seq_lens: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
                enable: Optional[torch.Tensor] = None, W: int = 0, num_splits: int = 1,
                workspace: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                shared_rows: int = 0) -> torch.Tensor:
    """Single-token attention.  q [B, Hq, d]; k/v [B, Hkv, S_max, d]; out [B, Hq, d].

    ``seq_lens`` (int32 [B], device) gives the number of valid keys per row
    (default: all S_max).  ``num_splits`` > 1 needs ``workspace`` (uint8, at
    least ``decode_workspace_bytes`` bytes).  ``shared_rows`` > 0: keys / values [0, shared_rows) are equal in
    every batch row (the caller's guarantee); they are read from row 0 (cram_attn_decode_shared, same results).
    """
    _check16("q", q, 3)
    _check16("k", k, 4, q)
    _check16("v", v, 4, q)
    B, Hq, d = q.shape
    _, Hkv, S, _ = k.shape
    if k.shape[0] != B or v.shape != k.shape or k.shape[3] != d:
        raise ValueError(f"shape mismatch q{tuple(q.shape)} k{tuple(k.shape)} v{tuple(v.shape)}")
    if seq_lens is not None and (seq_lens.dtype != torch.int32 or seq_lens.shape != (B,) or not seq_lens.is_cuda):
        raise ValueError("seq_lens must be a device int32 [B] tensor")
    if out is None:
        out = torch.empty((B, Hq, d), dtype=q.dtype, device=q.device)
    bp, bsb, ep, esb, W = _bias_args(bias, enable, B, Hq, W)
    lib = _lib.load()
    ws_ptr, ws_bytes = None, 0
    if num_splits > 1:
        need = decode_workspace_bytes(B, Hq, d, num_splits)
        if workspace is None:
            workspace = torch.empty(need, dtype=torch.uint8, device=q.device)
        ws_ptr, ws_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
    if shared_rows < 0 or shared_rows > S:
        raise ValueError("shared_rows must be in [0, S_max]")
    code = lib.cram_attn_decode_shared(
        q.data_ptr(), q.stride(0), q.stride(1),
        k.data_ptr(), k.stride(0), k.stride(1), k.stride(2),
        v.data_ptr(), v.stride(0), v.stride(1), v.stride(2),
        out.data_ptr(), out.stride(0), out.stride(1),
        B, Hq, Hkv, S, _ptr(seq_lens), d, float(scale),
        bp, bsb, ep, esb, W, int(shared_rows), int(num_splits), ws_ptr, ws_bytes, _dt(q), _stream(q.device))
    _lib.check(code, "cram_attn_decode_shared")
    return out


def answer_logits(hidden: torch.Tensor, w_lm: torch.Tensor, ids: torch.Tensor, *, round_logits: bool = False,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[i] = <hidden[i], w_lm[ids[i]]> in fp32, rounded to the model dtype first if ``round_logits``.
    hidden [n, D], w_lm [V, D] (bf16 or fp16, same dtype), ids int32 [n]."""
    _check16("hidden", hidden, 2)
    _check16("w_lm", w_lm, 2, hidden)
    n, D = hidden.shape
    if w_lm.shape[1] != D or ids.dtype != torch.int32 or ids.shape != (n,):
        raise ValueError("answer_logits: hidden [n, D], w_lm [V, D], ids int32 [n]")
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=hidden.device)
    lib = _lib.load()
    code = lib.cram_answer_logits(hidden.data_ptr(), hidden.stride(0), w_lm.data_ptr(), w_lm.stride(0),
                                  ids.data_ptr(), n, D, int(bool(round_logits)), out.data_ptr(), _dt(hidden),
                                  _stream(hidden.device))
    _lib.check(code, "cram_answer_logits")
    return out


def _rows2d(t: torch.Tensor, name: str) -> torch.Tensor:
    """View [..., C] with contiguous last dim as rows (returns the 2-D view; raises if not row-uniform)."""
    if t.stride(-1) != 1:
        raise ValueError(f"{name} must have a contiguous last dimension")
    if t.dim() == 2:
        return t
    try:
        return t.view(-1, t.shape[-1])
    except RuntimeError:
        raise ValueError(f"{name} rows are not uniformly strided") from None


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
            h_out: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None):
    """LlamaRMSNorm(x [+ residual]).  Returns y, or (h, y) when residual is given (h = x + residual)."""
    _check16("w", w, 1)
    _check16("x", x, x.dim(), w)
    x2 = _rows2d(x, "x")
    rows, D = x2.shape
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    y2 = _rows2d(out, "out")
    r2 = h2 = None
    if residual is not None:
        r2 = _rows2d(residual, "residual")
        if h_out is None:
            h_out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        h2 = _rows2d(h_out, "h_out")
    code = _lib.load().cram_rmsnorm(x2.data_ptr(), x2.stride(0), _ptr(r2), r2.stride(0) if r2 is not None else 0,
                                    _ptr(h2), h2.stride(0) if h2 is not None else 0, w.data_ptr(), y2.data_ptr(),
                                    y2.stride(0), rows, D, float(eps), _dt(x), _stream(x.device))
    _lib.check(code, "cram_rmsnorm")
    return (h_out, out) if residual is not None else out


def rope_inplace(qkv: torch.Tensor, heads: int, head_dim: int, cos: torch.Tensor, sin: torch.Tensor, T: int,
                 pos: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Rotate the first `heads` heads of every row of the fused QKV buffer in place (apply_rotary_pos_emb)."""
    y2 = _rows2d(qkv, "qkv")
    _dt(qkv)
    if cos.dtype != qkv.dtype or sin.dtype != qkv.dtype or cos.shape != sin.shape or cos.stride(-1) != 1:
        raise ValueError("cos/sin must be [P, d] tables of the QKV buffer's dtype")
    if pos is not None and (pos.dtype != torch.int64 or pos.numel() != y2.shape[0]):
        raise ValueError("pos must be int64 with one entry per row")
    code = _lib.load().cram_rope_inplace(y2.data_ptr(), y2.stride(0), y2.shape[0], int(T), int(heads), int(head_dim),
                                         cos.data_ptr(), sin.data_ptr(), cos.stride(0), _ptr(pos), _dt(qkv),
                                         _stream(qkv.device))
    _lib.check(code, "cram_rope_inplace")
    return qkv


def rope_split(qkv: torch.Tensor, hq: int, hkv: int, head_dim: int, cos: torch.Tensor, sin: torch.Tensor, T: int,
               kout: torch.Tensor, vout: torch.Tensor, row0: int, pos: Optional[torch.Tensor] = None,
               dst_b: Optional[torch.Tensor] = None, keep_k: bool = False) -> None:
    """RoPE over a fused q | k | v row buffer: q rotated in place, k rotated into kout (and kept in place too if
    ``keep_k``) and v copied into vout.  kout/vout are [B, S, hkv, head_dim] views with any strides (e.g. the
    decode cache [B, hkv, S, d] transposed).  Buffer row r goes to kout[r // T, row0 + r % T] (B * T rows), or,
    with ``dst_b`` (int64 per row, device), to kout[dst_b[r], row0 + pos[r]]: the caller guarantees
    dst_b < B and row0 + pos < S."""
    y2 = _rows2d(qkv, "qkv")
    dt = _dt(qkv)
    rows = y2.shape[0]
    if cos.dtype != qkv.dtype or sin.dtype != qkv.dtype or cos.shape != sin.shape or cos.stride(-1) != 1:
        raise ValueError("cos/sin must be [P, d] tables of the QKV buffer's dtype")
    if pos is not None and (pos.dtype != torch.int64 or pos.numel() != rows):
        raise ValueError("pos must be int64 with one entry per row")
    if dst_b is not None and (pos is None or dst_b.dtype != torch.int64 or dst_b.numel() != rows
                              or dst_b.device != qkv.device):
        raise ValueError("dst_b needs pos and must be a device int64 tensor with one entry per row")
    for t in (kout, vout):
        if (t.dtype != qkv.dtype or t.device != qkv.device or t.dim() != 4 or tuple(t.shape[2:]) != (hkv, head_dim)
                or t.stride(3) != 1):
            raise ValueError("kout/vout must be [B, S, hkv, head_dim] views with a contiguous last dimension")
        if dst_b is None and (t.shape[0] * T != rows or row0 + T > t.shape[1]):
            raise ValueError("kout/vout must hold B = rows / T sequences of at least row0 + T rows")
    if kout.stride()[:3] != vout.stride()[:3]:
        raise ValueError("kout and vout must share their strides")
    code = _lib.load().cram_rope_split(y2.data_ptr(), y2.stride(0), rows, int(T), int(hq), int(hkv), int(head_dim),
                                       cos.data_ptr(), sin.data_ptr(), cos.stride(0), _ptr(pos), kout.data_ptr(),
                                       vout.data_ptr(), kout.stride(0), kout.stride(2), kout.stride(1), int(row0),
                                       _ptr(dst_b), int(bool(keep_k)), dt, _stream(qkv.device))
    _lib.check(code, "cram_rope_split")


def silu_mul(gu: torch.Tensor, F: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """rnd(silu(gu[..., :F])) * gu[..., F:2F] (LlamaMLP activation), bf16 or fp16."""
    _dt(gu)
    g2 = _rows2d(gu, "gu")
    if out is None:
        out = torch.empty(gu.shape[:-1] + (F,), dtype=gu.dtype, device=gu.device)
    y2 = _rows2d(out, "out")
    code = _lib.load().cram_silu_mul(g2.data_ptr(), g2.stride(0), y2.data_ptr(), y2.stride(0), g2.shape[0], int(F),
                                     _dt(gu), _stream(gu.device))
    _lib.check(code, "cram_silu_mul")
    return out


GEMM_STORE = 0      # CRAM_GEMM_STORE
GEMM_SILU_MUL = 1   # CRAM_GEMM_SILU_MUL
GEMM_SILU_MUL_CAT = 2   # CRAM_GEMM_SILU_MUL_CAT


def interleave_gate_up(wgu: torch.Tensor, F: int) -> torch.Tensor:
    """[gate; up] rows ([2F, K], gate_proj then up_proj) -> rows interleaved in blocks of 32 (64j..64j+31 = gate
    32j.., 64j+32..64j+63 = up 32j..), the weight layout of cram_gemm's SiLU-mul epilogue."""
    if wgu.dim() != 2 or wgu.shape[0] != 2 * F or F % 32:
        raise ValueError(f"gate/up weight must be [2F, K] with F % 32 == 0, got {tuple(wgu.shape)}, F={F}")
    K = wgu.shape[1]
    return torch.stack([wgu[:F].reshape(F // 32, 32, K), wgu[F:].reshape(F // 32, 32, K)], 1).reshape(2 * F, K)


def gemm(x: torch.Tensor, w: torch.Tensor, epilogue: int = GEMM_STORE, out: Optional[torch.Tensor] = None,
         name: str = "cram_gemm", residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x [..., K] @ w[N, K]^T on the hand-written MFMA GEMM (cram_gemm); GEMM_SILU_MUL takes an interleaved gate/up
    weight (interleave_gate_up) and returns the MLP activation [..., N/2].  residual [..., N] (GEMM_STORE only):
    returns residual + x @ w^T with the add in the epilogue (cram_gemm_residual; `out` may be residual itself)."""
    _dt(x)
    if w.dtype != x.dtype or w.dim() != 2 or w.stride(1) != 1:
        raise ValueError("w must be a [N, K] row-major weight of x's dtype")
    x2 = _rows2d(x, "x")
    M, K = x2.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"K mismatch: x {K}, w {w.shape[1]}")
    nout = N if epilogue == GEMM_STORE else N // 2
    if out is None:
        out = torch.empty(x.shape[:-1] + (nout,), dtype=x.dtype, device=x.device)
    o2 = _rows2d(out, "out")
    if residual is not None:
        if epilogue != GEMM_STORE or residual.dtype != x.dtype or residual.shape[-1] != N:
            raise ValueError("residual must be a [..., N] tensor of x's dtype (GEMM_STORE only)")
        r2 = _rows2d(residual, "residual")
        if r2.shape[0] != M:
            raise ValueError(f"residual has {r2.shape[0]} rows, x has {M}")
    rbytes = 0 if residual is None else 2.0 * M * N
    ev = (TIMER.record(name, 2.0 * M * N * K, 2.0 * (M * K + N * K + M * nout) + rbytes, x.device)
          if TIMER.enabled else None)
    if residual is None:
        code = _lib.load().cram_gemm(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), o2.data_ptr(),
                                     o2.stride(0), M, N, K, int(epilogue), _dt(x), _stream(x.device))
        _lib.check(code, "cram_gemm")
    else:
        code = _lib.load().cram_gemm_residual(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), r2.data_ptr(),
                                              r2.stride(0), o2.data_ptr(), o2.stride(0), M, N, K, _dt(x),
                                              _stream(x.device))
        _lib.check(code, "cram_gemm_residual")
    if ev is not None:
        ev.record(torch.cuda.current_stream(x.device))
    return out


def gemm_rope(x: torch.Tensor, w: torch.Tensor, hq: int, hkv: int, head_dim: int, cos: torch.Tensor,
              sin: torch.Tensor, T: int, rows: Optional[int] = None, kout: Optional[torch.Tensor] = None,
              vout: Optional[torch.Tensor] = None, row0: int = 0, pos: Optional[torch.Tensor] = None,
              dst_b: Optional[torch.Tensor] = None, keep_k: bool = False, out: Optional[torch.Tensor] = None,
              pos0: int = 0, bias: Optional[torch.Tensor] = None, name: str = "cram_gemm") -> torch.Tensor:
    """The q | k | v projection x @ w^T with RoPE in the GEMM epilogue (cram_gemm_rope, the 4-wave kernel; bf16 or
    fp16, head_dim 128, optional q/k/v bias).  Without kout / vout: ``rope_inplace`` over the q and k heads of the result (T, pos as
    there; without pos the table row is pos0 + m % T).  With them: ``rope_split`` into kout / vout ([B, S, hkv, d]
    views, row0, pos, dst_b, keep_k as there),
    for the first ``rows`` rows of x (default all; rows beyond are GEMM padding).  Returns the [M, N] buffer: q
    rotated; k rotated and v as computed unless kout is given without keep_k (then those columns are not written).
    bias [N] (Qwen2's q/k/v): the projection is rnd(x @ w^T + bias) before RoPE, as F.linear rounds it."""
    _dt(x)
    if w.dtype != x.dtype or w.dim() != 2 or w.stride(1) != 1:
        raise ValueError("w must be a [N, K] row-major weight of x's dtype")
    x2 = _rows2d(x, "x")
    M, K = x2.shape
    N = w.shape[0]
    if w.shape[1] != K or N != (hq + 2 * hkv) * head_dim:
        raise ValueError(f"w must be [(hq + 2 hkv) * head_dim, K], got {tuple(w.shape)}")
    rows = M if rows is None else int(rows)
    if cos.dtype != x.dtype or sin.dtype != x.dtype or cos.shape != sin.shape or cos.stride(-1) != 1:
        raise ValueError("cos/sin must be [P, d] tables of x's dtype")
    if pos is not None and (pos.dtype != torch.int64 or pos.numel() < rows or pos.device != x.device):
        raise ValueError("pos must be a device int64 tensor with one entry per row")
    if (kout is None) != (vout is None):
        raise ValueError("kout and vout go together")
    if kout is not None:
        for t in (kout, vout):
            if (t.dtype != x.dtype or t.device != x.device or t.dim() != 4 or tuple(t.shape[2:]) != (hkv, head_dim)
                    or t.stride(3) != 1):
                raise ValueError("kout/vout must be [B, S, hkv, head_dim] views with a contiguous last dimension")
        if kout.stride()[:3] != vout.stride()[:3]:
            raise ValueError("kout and vout must share their strides")
        if dst_b is None and (rows % T or rows // T > kout.shape[0] or row0 + T > kout.shape[1]):
            raise ValueError("kout/vout must hold rows / T sequences of at least row0 + T rows")
        if dst_b is not None and (pos is None or dst_b.dtype != torch.int64 or dst_b.numel() < rows
                                  or dst_b.device != x.device):
            raise ValueError("dst_b needs pos and must be a device int64 tensor with one entry per row")
    if bias is not None and (bias.dtype != x.dtype or bias.numel() != N or not bias.is_contiguous()
                             or bias.device != x.device):
        raise ValueError("bias must be a contiguous [N] device tensor of x's dtype")
    if out is None:
        out = torch.empty(x.shape[:-1] + (N,), dtype=x.dtype, device=x.device)
    o2 = _rows2d(out, "out")
    ev = TIMER.record(name, 2.0 * M * N * K, 2.0 * (M * K + N * K + M * N), x.device) if TIMER.enabled else None
    st = (0, 0, 0) if kout is None else (kout.stride(0), kout.stride(2), kout.stride(1))
    code = _lib.load().cram_gemm_rope(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), _ptr(bias), o2.data_ptr(),
                                      o2.stride(0), M, K, rows, int(T), int(hq), int(hkv), int(head_dim),
                                      cos.data_ptr(), sin.data_ptr(), cos.stride(0), _ptr(pos), int(pos0), _ptr(kout),
                                      _ptr(vout), st[0], st[1], st[2], int(row0), _ptr(dst_b), int(bool(keep_k)),
                                      _dt(x), _stream(x.device))
    _lib.check(code, "cram_gemm_rope")
    if ev is not None:
        ev.record(torch.cuda.current_stream(x.device))
    return out


def gemm_small(x: torch.Tensor, w: torch.Tensor, splits: int = 1, epilogue: int = GEMM_STORE,
               bias: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
               out: Optional[torch.Tensor] = None, name: str = "cram_gemm_small") -> torch.Tensor:
    """x [..., K] @ w[N, K]^T (+ bias) on the decode-step GEMM (cram_gemm_small: 128 x 128 tiles, a four-deep LDS
    ring; few rows); GEMM_SILU_MUL takes the interleaved gate/up weight (interleave_gate_up) and returns [..., N/2].
    splits > 1 cuts K into ranges combined in order through `workspace` (a uint8 device tensor of
    >= gemm_splitk_workspace_bytes(M, N, splits); allocated here when None, pass one for hipGraph capture)."""
    _dt(x)
    if w.dtype != x.dtype or w.dim() != 2 or w.stride(1) != 1:
        raise ValueError("w must be a [N, K] row-major weight of x's dtype")
    x2 = _rows2d(x, "x")
    M, K = x2.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"K mismatch: x {K}, w {w.shape[1]}")
    if bias is not None and (bias.dtype != x.dtype or bias.numel() != N or not bias.is_contiguous()):
        raise ValueError("bias must be a contiguous [N] tensor of x's dtype")
    nout = N if epilogue == GEMM_STORE else N // 2
    if out is None:
        out = torch.empty(x.shape[:-1] + (nout,), dtype=x.dtype, device=x.device)
    o2 = _rows2d(out, "out")
    if splits > 1 and workspace is None:
        workspace = torch.empty(gemm_splitk_workspace_bytes(M, N, splits), dtype=torch.uint8, device=x.device)
    ev = (TIMER.record(name, 2.0 * M * N * K, 2.0 * (M * K + N * K + M * nout), x.device) if TIMER.enabled else None)
    code = _lib.load().cram_gemm_small(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), _ptr(bias),
                                       o2.data_ptr(), o2.stride(0), M, N, K, int(splits), int(epilogue),
                                       _ptr(workspace), 0 if workspace is None else workspace.numel(), _dt(x),
                                       _stream(x.device))
    _lib.check(code, "cram_gemm_small")
    if ev is not None:
        ev.record(torch.cuda.current_stream(x.device))
    return out


def gemm_splitk_workspace_bytes(M: int, N: int, splits: int) -> int:
    return int(_lib.load().cram_gemm_splitk_workspace_size(int(M), int(N), int(splits)))


def gemm_splitk(x: torch.Tensor, w: torch.Tensor, splits: int, epilogue: int = GEMM_STORE,
                bias: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, name: str = "cram_gemm_splitk",
                residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x [..., K] @ w[N, K]^T (+ bias) with K cut into `splits` ranges (cram_gemm_splitk: the decode step's skinny
    projections); GEMM_SILU_MUL_CAT takes the checkpoint's [gate; up] weight and returns the MLP activation
    [..., N/2].  workspace: a uint8 device tensor of >= gemm_splitk_workspace_bytes(M, N, splits) (allocated here
    when None; pass one for hipGraph capture).  residual [..., N] (GEMM_STORE, no bias): returns residual + x @ w^T
    with the add in the combine (cram_gemm_splitk_residual; `out` may be residual itself)."""
    _dt(x)
    if w.dtype != x.dtype or w.dim() != 2 or w.stride(1) != 1:
        raise ValueError("w must be a [N, K] row-major weight of x's dtype")
    x2 = _rows2d(x, "x")
    M, K = x2.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"K mismatch: x {K}, w {w.shape[1]}")
    if bias is not None and (bias.dtype != x.dtype or bias.numel() != N or not bias.is_contiguous()):
        raise ValueError("bias must be a contiguous [N] tensor of x's dtype")
    nout = N if epilogue == GEMM_STORE else N // 2
    if out is None:
        out = torch.empty(x.shape[:-1] + (nout,), dtype=x.dtype, device=x.device)
    o2 = _rows2d(out, "out")
    need = gemm_splitk_workspace_bytes(M, N, splits)
    if workspace is None:
        workspace = torch.empty(need, dtype=torch.uint8, device=x.device)
    if residual is not None:
        if epilogue != GEMM_STORE or bias is not None or residual.dtype != x.dtype or residual.shape[-1] != N:
            raise ValueError("residual must be a [..., N] tensor of x's dtype (GEMM_STORE, no bias)")
        r2 = _rows2d(residual, "residual")
        if r2.shape[0] != M:
            raise ValueError(f"residual has {r2.shape[0]} rows, x has {M}")
    rbytes = 0 if residual is None else 2.0 * M * N
    ev = (TIMER.record(name, 2.0 * M * N * K, 2.0 * (M * K + N * K + M * nout) + rbytes, x.device)
          if TIMER.enabled else None)
    if residual is None:
        code = _lib.load().cram_gemm_splitk(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), o2.data_ptr(),
                                            o2.stride(0), M, N, K, int(splits), int(epilogue),
                                            None if bias is None else bias.data_ptr(), workspace.data_ptr(),
                                            workspace.numel(), _dt(x), _stream(x.device))
        _lib.check(code, "cram_gemm_splitk")
    else:
        code = _lib.load().cram_gemm_splitk_residual(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0),
                                                     r2.data_ptr(), r2.stride(0), o2.data_ptr(), o2.stride(0), M, N, K,
                                                     int(splits), workspace.data_ptr(), workspace.numel(), _dt(x),
                                                     _stream(x.device))
        _lib.check(code, "cram_gemm_splitk_residual")
    if ev is not None:
        ev.record(torch.cuda.current_stream(x.device))
    return out
