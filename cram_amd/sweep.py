"""Head-batched indirect-effect (IE) sweep — the MI355X form of Find_Best_Heads.cal_logits.

Reference (re_weighting.py:152-175): for one question, one un-hooked forward
gives ori = sum_k logits[0, -n+k, a_k]; then for every (layer l, head h) one
full forward with the credibility mask on head h of layer l only gives cur;
IE[l][h] = ori - cur.  That is 1 + L*H full forwards, each with full-vocab
logits and a host sync.

Here, per question:
  1. one baseline forward caches, for every layer l, the layer input h_l, the
     roped q/k/v and the un-biased attention output A_l;
  2. for every layer l, ONE all-heads-biased attention call gives each head's
     perturbed output; variant h = A_l with head h's slice replaced, so the H
     variants of layer l are a batch of H sequences that share h_l;
  3. the batch runs o_proj + MLP of layer l and the unchanged layers l+1..L-1
     (plain causal attention), the last layer only for the n answer rows;
  4. answer logits come from the fp32 gather-dot kernel (no full vocab);
  5. IE stays on the device; one host copy per question (or one all-gather).
Noise cancellation: in the reference, ori and cur share bit-identical arithmetic
for every layer below the hooked one (re_weighting.py:159 vs :169).  Here each
layer's batch also carries one UN-perturbed variant, and IE[l, h] = sum over the
un-perturbed row - sum over variant h, so the two sides again share their
rounding everywhere except in the perturbed computation (the layer-l batch
shape differs from the batch-1 baseline, so re-using the baseline's ori would
leave uncorrelated bf16 rounding in the difference).
Work per question: L*H*(L-1)/2 + ... layer-forwards instead of (1 + L*H) * L.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import gemm_tune, ops
from .bias import CredibilityBias
from .engine import CrAMEngine, padded_rows


class QuestionCache:
    """Baseline-forward state of one question (device tensors)."""

    def __init__(self):
        self.h_in = []     # layer input  [1, T, D]
        self.q = []        # roped q      [1, T, Hq, d]
        self.k = []        # roped k      [1, T, Hkv, d]
        self.v = []        # v            [1, T, Hkv, d]
        self.a = []        # un-biased attention output [1, T, Hq, d]


@torch.no_grad()
def baseline(eng: CrAMEngine, ids: torch.Tensor, n_ans: int, keep: bool = True):
    """Un-hooked forward; returns (final hidden of the last n rows [n, D], QuestionCache)."""
    sp = eng.spec
    T = ids.shape[-1]
    cos, sin = eng.rope_tables(T)
    h = eng.embed[ids.view(1, T)]
    qc = QuestionCache()
    L = sp.num_layers
    for l in range(L):
        lw = eng.layers[l]
        x = eng.rmsnorm(h, lw.ln1)
        q, k, v = eng.qkv(x, lw, cos, sin)
        a = eng.attention(q, k, v)
        if keep:
            qc.h_in.append(h)
            qc.q.append(q)
            qc.k.append(k)
            qc.v.append(v)
            qc.a.append(a)
        if l == L - 1:
            a = a[:, -n_ans:]
            h = h[:, -n_ans:]
        h, x2 = eng.add_rmsnorm(ops.linear(a.flatten(-2), lw.wo), h, lw.ln2)
        h = h + eng.mlp(x2, lw)
    return eng.rmsnorm(h, eng.norm)[0], qc


def first_biased_row(bias: torch.Tensor, W: int) -> int:
    """p0 = first key position whose credibility bias is not 0.  Query rows before p0 see no biased key, so
    (causal attention) they are identical in every variant of every layer: the sweep computes rows >= p0
    only and takes the K/V of rows < p0 from the baseline forward."""
    nz = torch.nonzero(bias[0, :W] != 0)
    return int(nz[0, 0]) if nz.numel() else W


@torch.no_grad()
def layer_variants(eng: CrAMEngine, qc: QuestionCache, l: int, bias: torch.Tensor, W: int, n_ans: int,
                   heads: Optional[torch.Tensor] = None, p0: int = 0) -> torch.Tensor:
    """Final hidden states [H'+1, n, D]: variants 'head heads[i] of layer l re-weighted', then the un-perturbed one.

    Rows < p0 (before the first biased key) are taken from the baseline instead of being recomputed per variant."""
    sp = eng.spec
    H = sp.num_heads
    heads = torch.arange(H, device=eng.device) if heads is None else heads
    Hv = heads.numel() + 1                                               # + the un-perturbed variant (last)
    T_full = qc.h_in[l].shape[1]
    L = sp.num_layers
    last = l == L - 1
    p0 = max(0, min(int(p0), T_full - n_ans))                           # the answer rows are always computed
    T = T_full - p0                                                     # suffix rows per variant
    enable = torch.ones((1, H), dtype=torch.uint8, device=eng.device)
    q, k, v = qc.q[l], qc.k[l], qc.v[l]
    rows = n_ans if last else T
    q = q[:, -rows:]
    a_bias = eng.attention(q, k, v, bias, enable, W)                   # [1, rows, Hq, d] every head biased
    a_base = qc.a[l][:, -rows:]
    M = Hv * rows
    Mp = M if last else padded_rows(M, sp)                              # GEMM rows: macro tile / measured table
    abuf = torch.empty((Mp, sp.q_size), dtype=eng.dtype, device=eng.device)
    x = abuf[:M].view(Hv, rows, H, sp.head_dim)
    x.copy_(a_base.expand(Hv, rows, H, sp.head_dim))                    # [Hv, rows, Hq, d]
    idx = torch.arange(Hv - 1, device=eng.device)
    x[idx, :, heads] = a_bias[0].permute(1, 0, 2)[heads]                # variant i <- biased head heads[i]
    lw = eng.layers[l]
    hin = torch.empty((Mp, sp.hidden), dtype=eng.dtype, device=eng.device)
    hin[:M].view(Hv, rows, sp.hidden).copy_(qc.h_in[l][:, -rows:].expand(Hv, rows, sp.hidden))
    h, x2 = eng.o_proj_norm(abuf, lw, hin)                             # [Mp, D]
    h, m = eng.mlp_residual(x2, lw, h)                                  # layer output h (+ m when deferred)
    if not last:
        cos, sin = eng.rope_tables(T_full)
        for l2 in range(l + 1, L):
            pre = None if p0 == 0 else (qc.k[l2][:, :p0], qc.v[l2][:, :p0])         # suffix row t at p0 + t
            h, m = eng.layer_rows(h, Hv, T, l2, cos, sin, out_rows=n_ans if l2 == L - 1 else None, delta=m,
                                  prefix=pre)
    rows = Hv * n_ans
    if m is None:
        y = ops.rmsnorm(h[:rows], eng.norm, sp.eps)
    else:
        _, y = ops.rmsnorm(m[:rows], eng.norm, sp.eps, residual=h[:rows])   # final norm of h + m
    return y.view(Hv, n_ans, sp.hidden)                                 # [Hv, n, D]


@torch.no_grad()
def ie_question(eng: CrAMEngine, ids: torch.Tensor, weight16: torch.Tensor, answer_ids: torch.Tensor,
                layers=None, round_logits: bool = False, skip_prefix: bool = True) -> torch.Tensor:
    """IE [len(layers), H] (fp32, device) for one question — the value cal_logits returns.

    ids [T'] (prompt + answer), weight16 fp16 [T'] (sweep scores), answer_ids [n]
    (standalone tokenisation, first id dropped: re_weighting.py:155).
    """
    with gemm_tune.pinned():
        return _ie_question(eng, ids, weight16, answer_ids, layers, round_logits, skip_prefix)


def _ie_question(eng, ids, weight16, answer_ids, layers, round_logits, skip_prefix):
    sp = eng.spec
    dev = eng.device
    ids = ids.to(dev).view(-1)
    n = int(answer_ids.numel())
    ans = answer_ids.to(dev, torch.int32).view(-1)
    cb = CredibilityBias.build([weight16.view(1, -1)], {}, sp.num_layers, sp.num_heads, dev, eng.dtype)
    _, qc = baseline(eng, ids, n)
    layers = range(sp.num_layers) if layers is None else layers
    out = torch.empty((len(layers), sp.num_heads), dtype=torch.float32, device=dev)
    H1 = sp.num_heads + 1
    ans_rep = ans.repeat(H1)
    p0 = first_biased_row(cb.bias, cb.W) if skip_prefix else 0
    for i, l in enumerate(layers):
        hv = layer_variants(eng, qc, l, cb.bias, cb.W, n, p0=p0)       # [H+1, n, D]
        sums = eng.answer_logits(hv.reshape(-1, sp.hidden), ans_rep, round_logits).view(H1, n).sum(1)
        out[i] = sums[-1] - sums[:-1]                                   # ori - cur
    return out


def sweep_flops(spec, T: int, n_ans: int, p0: int = 0, layers=None) -> float:
    """Algorithmic GEMM+attention flops of ie_question(layers=...) (for roofline accounting): one baseline
    forward plus the suffix work of every swept layer; p0 = skipped prefix rows."""
    L, H, d, D = spec.num_layers, spec.num_heads, spec.head_dim, spec.hidden

    def attn(tq, s):   # tq queries at positions s-tq .. s-1, causal
        vis = tq * (s - tq) + tq * (tq + 1) / 2.0
        return 4.0 * d * spec.num_heads * vis

    lay = lambda t: spec.layer_flops(t)
    qkv_frac = (spec.q_size + 2 * spec.kv_size) * D / ((spec.q_size + 2 * spec.kv_size) * D + spec.q_size * D
                                                      + 3 * D * spec.intermediate)
    p0 = max(0, min(p0, T - n_ans))
    Ts = T - p0
    f = 0.0
    # baseline: L-1 full layers + last layer (qkv over T, rest over n)
    f += (L - 1) * (lay(T) + attn(T, T)) + qkv_frac * lay(T) + (1 - qkv_frac) * lay(n_ans) + attn(n_ans, T)
    for l in (range(L) if layers is None else layers):
        last = l == L - 1
        rows = n_ans if last else Ts
        f += attn(rows, T)                                              # all-heads biased attention
        f += (H + 1) * (1 - qkv_frac) * lay(rows)                       # o_proj + MLP of layer l, H+1 variants
        for l2 in range(l + 1, L):
            if l2 == L - 1:
                f += (H + 1) * (qkv_frac * lay(Ts) + (1 - qkv_frac) * lay(n_ans) + attn(n_ans, T))
            else:
                f += (H + 1) * (lay(Ts) + attn(Ts, T))
    return f
