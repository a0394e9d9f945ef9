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
for every layer below the hooked one (re_weighting.py:159 vs :169).  In the
row-exact mode (the default since round 6) that holds by
construction: the baseline forward and the variant batches run every projection on
the same kernel (the 4-wave GEMM whatever the row count, no split-K tail, whose
per-element accumulation order does not depend on M or on the row's place), the
baseline's attention over the suffix rows [p0, T) as one call of the shape the
variants' calls have, so an un-perturbed row computes the same bits in the baseline
as in any variant batch, and IE[l, h] = ori(baseline) - sum over variant h.  Where
the fused kernels do not apply (the CPU stand-ins, widths the epilogues do not take;
CRAM_SWEEP_ROW_EXACT=0) each layer's batch carries one un-perturbed variant (first)
and IE[l, h] = its sum - variant h's, so ori and cur round alike.
Work per question: L*H*(L-1)/2 + ... layer-forwards instead of (1 + L*H) * L.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch

from . import gemm_tune, ops
from .bias import CredibilityBias
from .engine import CrAMEngine, padded_rows

# Row-exact sweep (the default since round 6; CRAM_SWEEP_ROW_EXACT=0 carries the un-perturbed variant in every batch):
# the baseline forward rounds every un-perturbed row as the variant batches do, so no batch carries an un-perturbed
# variant (1/33 of the work).  It passes the multi-question full-grid bars of tests/test_fullsize_ie_gpu.py over 13
# NQ questions (RMS error vs the float32 truth 0.943x the reference algorithm's own, k = 894 overlap -1.7 against a
# -13.8 bar; the carried-variant mode: 0.930x, -2.2), +1.7 % heads/s (profiles/r06/)
ROW_EXACT = os.environ.get("CRAM_SWEEP_ROW_EXACT", "1") == "1"
# CRAM_ROW_EXACT_TAIL_SPLIT=1: the variant batches keep the split-K tail of o_proj / down_proj (+0.5 %, but the tail's
# rows then sum their K ranges in another order than the baseline's: not row-exact for those rows)
EXACT_TAIL_SPLIT = os.environ.get("CRAM_ROW_EXACT_TAIL_SPLIT", "0") == "1"
# consecutive swept layers whose variant batches share one growing batch (group_variants; bit-identical IE in the
# row-exact mode): groups of 4 ran 222.0 heads/s against 218.4 for a batch per layer (2: 221.0, 8: 220.6, whose
# ~230k-row buffers cost the allocator more than the fuller waves return), same box, profiles/r06/group/;
# CRAM_SWEEP_GROUP=1 runs a batch per layer (A/B)
SWEEP_GROUP = int(os.environ.get("CRAM_SWEEP_GROUP", "4"))


class QuestionCache:
    """Baseline-forward state of one question (device tensors)."""

    def __init__(self):
        self.h_in = []     # layer input  [1, T, D]
        self.q = []        # roped q      [1, T, Hq, d]
        self.k = []        # roped k      [1, T, Hkv, d]
        self.v = []        # v            [1, T, Hkv, d]
        self.a = []        # un-biased attention output [1, T, Hq, d] (last layer, row-exact: the last n rows)
        self.exact = False  # built row-exact (baseline()): the sweep needs no un-perturbed variant


def row_exact(eng: CrAMEngine) -> bool:
    """True when the sweep's un-perturbed rows compute the same bits in the baseline forward as in the variant
    batches (every projection on the fused 4-wave kernels: a CUDA engine at 16-bit widths the fused epilogues
    take); the sweep then drops the per-layer un-perturbed variant."""
    if not ROW_EXACT or eng.device.type != "cuda":
        return False
    x = torch.empty((1, eng.spec.hidden), device="meta")
    with _modes(eng, True, False):
        return eng._fused_residual_ok(x) and eng._fused_qkv_ok(x, eng.layers[0])


@contextlib.contextmanager
def _modes(eng: CrAMEngine, fused_any_rows: bool, no_tail_split: bool):
    prev = eng.fused_any_rows, eng.no_tail_split
    eng.fused_any_rows, eng.no_tail_split = fused_any_rows, no_tail_split
    try:
        yield
    finally:
        eng.fused_any_rows, eng.no_tail_split = prev


@torch.no_grad()
def baseline(eng: CrAMEngine, ids: torch.Tensor, n_ans: int, keep: bool = True, p0: int = 0):
    """Un-hooked forward; returns (final hidden of the last n rows [n, D], QuestionCache).

    Row-exact (row_exact(eng)): the fused projections at any row count, and each layer's attention as two calls,
    rows [0, p0) and rows [p0, T) (the last layer: the last n rows) -- the query blocks of the variants' calls."""
    sp = eng.spec
    T = ids.shape[-1]
    cos, sin = eng.rope_tables(T)
    h = eng.embed[ids.view(1, T)]
    qc = QuestionCache()
    L = sp.num_layers
    exact = row_exact(eng)
    p0 = max(0, min(int(p0), T - n_ans))
    with _modes(eng, exact, exact):
        for l in range(L):
            lw = eng.layers[l]
            x = eng.rmsnorm(h, lw.ln1)
            q, k, v = eng.qkv(x, lw, cos, sin)
            last = l == L - 1
            if not exact:
                a = eng.attention(q, k, v)
            elif last:
                a = eng.attention(q[:, -n_ans:], k, v)
            else:
                a = torch.empty((1, T, sp.num_heads, sp.head_dim), dtype=eng.dtype, device=eng.device)
                if p0 > 0:
                    ops.attn_prefill(q[:, :p0].transpose(1, 2), k[:, :p0].transpose(1, 2), v[:, :p0].transpose(1, 2),
                                     scale=eng.scale, out=a[:, :p0])
                ops.attn_prefill(q[:, p0:].transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale=eng.scale,
                                 out=a[:, p0:])
            if keep:
                qc.h_in.append(h)
                qc.q.append(q)
                qc.k.append(k)
                qc.v.append(v)
                qc.a.append(a)
            if last:
                a = a[:, -n_ans:]
                h = h[:, -n_ans:]
            if exact:
                rows = a.shape[1]
                h2, x2 = eng.o_proj_norm(a.reshape(rows, sp.q_size), lw, h.reshape(rows, sp.hidden))
                h, _ = eng.mlp_residual(x2, lw, h2)
                h = h.view(1, rows, sp.hidden)
            else:
                h, x2 = eng.add_rmsnorm(ops.linear(a.flatten(-2), lw.wo), h, lw.ln2)
                h = h + eng.mlp(x2, lw)
        qc.exact = exact
        return eng.rmsnorm(h, eng.norm)[0], qc


def first_biased_row(bias: torch.Tensor, W: int) -> int:
    """p0 = first key position whose credibility bias is not 0.  Query rows before p0 see no biased key, so
    (causal attention) they are identical in every variant of every layer: the sweep computes rows >= p0
    only and takes the K/V of rows < p0 from the baseline forward."""
    nz = torch.nonzero(bias[0, :W] != 0)
    return int(nz[0, 0]) if nz.numel() else W


@torch.no_grad()
def layer_variants(eng: CrAMEngine, qc: QuestionCache, l: int, bias: torch.Tensor, W: int, n_ans: int,
                   heads: Optional[torch.Tensor] = None, p0: int = 0, with_base: Optional[bool] = None):
    """Final hidden states [(1 +) H', n, D]: (with_base; default: when the cache is not row-exact) the un-perturbed
    variant first, then the variants 'head heads[i] of layer l re-weighted'.  The un-perturbed variant leads so that
    its rows sit in the whole waves of every projection launch, away from the split-K tail (engine._gemm_residual).

    Rows < p0 (before the first biased key) are taken from the baseline instead of being recomputed per variant."""
    sp = eng.spec
    H = sp.num_heads
    heads = torch.arange(H, device=eng.device) if heads is None else heads
    if with_base is None:
        with_base = not qc.exact
    b0 = 1 if with_base else 0
    Hv = heads.numel() + b0                                             # (+ the un-perturbed variant, first)
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
    no_tail = qc.exact and not EXACT_TAIL_SPLIT
    Mp = M if last else padded_rows(M, sp, no_tail)                     # GEMM rows: macro tile / measured table
    abuf = torch.empty((Mp, sp.q_size), dtype=eng.dtype, device=eng.device)
    x = abuf[:M].view(Hv, rows, H, sp.head_dim)
    x.copy_(a_base.expand(Hv, rows, H, sp.head_dim))                    # [Hv, rows, Hq, d]
    idx = torch.arange(b0, Hv, device=eng.device)
    x[idx, :, heads] = a_bias[0].permute(1, 0, 2)[heads]                # variant b0 + i <- biased head heads[i]
    lw = eng.layers[l]
    hin = torch.empty((Mp, sp.hidden), dtype=eng.dtype, device=eng.device)
    hin[:M].view(Hv, rows, sp.hidden).copy_(qc.h_in[l][:, -rows:].expand(Hv, rows, sp.hidden))
    # row-exact: the variant batches run every row on the 4-wave kernel too (no split-K tail), so every variant row
    # rounds as the baseline's does (the tail's rows used to sum their K ranges in another order);
    # CRAM_ROW_EXACT_TAIL_SPLIT=1 keeps the split-K tail in the variant batches (A/B of its cost)
    with _modes(eng, qc.exact, qc.exact and not EXACT_TAIL_SPLIT):
        h, x2 = eng.o_proj_norm(abuf, lw, hin)                         # [Mp, D]
        h, m = eng.mlp_residual(x2, lw, h)                              # layer output h (+ m when deferred)
        if not last:
            cos, sin = eng.rope_tables(T_full)
            for l2 in range(l + 1, L):
                pre = None if p0 == 0 else (qc.k[l2][:, :p0], qc.v[l2][:, :p0])     # suffix row t at p0 + t
                h, m = eng.layer_rows(h, Hv, T, l2, cos, sin, out_rows=n_ans if l2 == L - 1 else None, delta=m,
                                      prefix=pre)
    rows = Hv * n_ans
    if m is None:
        y = ops.rmsnorm(h[:rows], eng.norm, sp.eps)
    else:
        _, y = ops.rmsnorm(m[:rows], eng.norm, sp.eps, residual=h[:rows])   # final norm of h + m
    return y.view(Hv, n_ans, sp.hidden)                                 # [Hv, n, D]


def _variant_inputs(eng: CrAMEngine, qc: QuestionCache, l: int, bias: torch.Tensor, W: int, T: int, b0: int):
    """The perturbed layer-l inputs of one variant batch over the suffix rows (the last T rows): attention output
    [Hv * T, q_size] (head h of variant b0 + h from the all-heads-biased call, the rest the baseline's) and the
    residual input [Hv * T, D]; Hv = H + b0 (b0 = 1: the un-perturbed variant first)."""
    sp = eng.spec
    H = sp.num_heads
    Hv = H + b0
    enable = torch.ones((1, H), dtype=torch.uint8, device=eng.device)
    a_bias = eng.attention(qc.q[l][:, -T:], qc.k[l], qc.v[l], bias, enable, W)        # [1, T, Hq, d]
    a = torch.empty((Hv * T, sp.q_size), dtype=eng.dtype, device=eng.device)
    x = a.view(Hv, T, H, sp.head_dim)
    x.copy_(qc.a[l][:, -T:].expand(Hv, T, H, sp.head_dim))
    heads = torch.arange(H, device=eng.device)
    x[heads + b0, :, heads] = a_bias[0].permute(1, 0, 2)
    hin = qc.h_in[l][:, -T:].expand(Hv, T, sp.hidden).reshape(Hv * T, sp.hidden)
    return a, hin


@torch.no_grad()
def group_variants(eng: CrAMEngine, qc: QuestionCache, ls, bias: torch.Tensor, W: int, n_ans: int, p0: int = 0,
                   with_base: Optional[bool] = None):
    """layer_variants for a run of consecutive layers ls (all below the last) in ONE growing batch: the variant batch
    of ls[0] starts at its layer; at each later layer of ls that layer's batch joins after the attention (its
    attention output is the perturbed one, the running sequences compute theirs), so o_proj, the MLP and every layer
    above run over all joined sequences in one launch each -- fewer launches and fuller waves of 256 x 256 tiles than
    one batch per layer.  Every kernel is row-independent (the 4-wave GEMM's per-element accumulation order does not
    depend on M or on the row's place; attention per sequence), so each variant's result is the one layer_variants
    gives (row-exact mode: bit for bit, tests/test_fullsize_ie_gpu.py).  Returns {l: [Hv, n, D]}."""
    sp = eng.spec
    L, H = sp.num_layers, sp.num_heads
    ls = list(ls)
    assert ls and all(b == a + 1 for a, b in zip(ls, ls[1:])) and ls[-1] < L - 1, ls
    if with_base is None:
        with_base = not qc.exact
    b0 = 1 if with_base else 0
    Hv = H + b0
    T_full = qc.h_in[ls[0]].shape[1]
    p0 = max(0, min(int(p0), T_full - n_ans))
    T = T_full - p0
    cos, sin = eng.rope_tables(T_full)
    h = m = None
    nseq = 0
    with _modes(eng, qc.exact, qc.exact and not EXACT_TAIL_SPLIT):
        for l2 in range(ls[0], L):
            pre = None if p0 == 0 else (qc.k[l2][:, :p0], qc.v[l2][:, :p0])
            join = _variant_inputs(eng, qc, l2, bias, W, T, b0) if l2 in ls else None
            if nseq == 0:                                               # the first batch: layer_variants' start
                lw = eng.layers[l2]
                M = Hv * T
                Mp = padded_rows(M, sp, eng.no_tail_split)
                abuf = torch.empty((Mp, sp.q_size), dtype=eng.dtype, device=eng.device)
                hin = torch.empty((Mp, sp.hidden), dtype=eng.dtype, device=eng.device)
                abuf[:M] = join[0]
                hin[:M] = join[1]
                h, x2 = eng.o_proj_norm(abuf, lw, hin)
                h, m = eng.mlp_residual(x2, lw, h)
            else:
                h, m = eng.layer_rows(h, nseq, T, l2, cos, sin, out_rows=n_ans if l2 == L - 1 else None, delta=m,
                                      prefix=pre, join=join)
            if join is not None:
                nseq += Hv
    rows = nseq * n_ans
    if m is None:
        y = ops.rmsnorm(h[:rows], eng.norm, sp.eps)
    else:
        _, y = ops.rmsnorm(m[:rows], eng.norm, sp.eps, residual=h[:rows])
    y = y.view(len(ls), Hv, n_ans, sp.hidden)
    return {l: y[i] for i, l in enumerate(ls)}


def sweep_groups(layers, num_layers: int, group: int):
    """Runs of at most `group` consecutive layers below the last (group_variants), the last layer alone."""
    out, run = [], []
    for l in sorted(layers):
        if l == num_layers - 1 or group <= 1:
            if run:
                out.append(run)
                run = []
            out.append([l])
            continue
        if run and (l != run[-1] + 1 or len(run) == group):
            out.append(run)
            run = []
        run.append(l)
    if run:
        out.append(run)
    return out


@torch.no_grad()
def ie_question(eng: CrAMEngine, ids: torch.Tensor, weight16: torch.Tensor, answer_ids: torch.Tensor,
                layers=None, round_logits: bool = False, skip_prefix: bool = True) -> torch.Tensor:
    """IE [len(layers), H] (fp32, device) for one question — the value cal_logits returns.

    ids [T'] (prompt + answer), weight16 fp16 [T'] (sweep scores), answer_ids [n]
    (standalone tokenisation, first id dropped: re_weighting.py:155).
    """
    with gemm_tune.pinned():
        return _ie_question(eng, ids, weight16, answer_ids, layers, round_logits, skip_prefix)


def _answer_sums(lg: torch.Tensor) -> torch.Tensor:
    """Row sums of [R, n] answer logits, left to right: the same fp32 additions whatever R (a reduction kernel's
    order may depend on the tensor's shape, and ori and cur must round alike)."""
    s = lg[:, 0].clone()
    for j in range(1, lg.shape[1]):
        s += lg[:, j]
    return s


def _ie_question(eng, ids, weight16, answer_ids, layers, round_logits, skip_prefix):
    sp = eng.spec
    dev = eng.device
    ids = ids.to(dev).view(-1)
    n = int(answer_ids.numel())
    ans = answer_ids.to(dev, torch.int32).view(-1)
    cb = CredibilityBias.build([weight16.view(1, -1)], {}, sp.num_layers, sp.num_heads, dev, eng.dtype)
    p0 = first_biased_row(cb.bias, cb.W) if skip_prefix else 0
    hf, qc = baseline(eng, ids, n, p0=p0)
    layers = range(sp.num_layers) if layers is None else layers
    out = torch.empty((len(layers), sp.num_heads), dtype=torch.float32, device=dev)
    H = sp.num_heads
    Hv = H if qc.exact else H + 1
    ans_rep = ans.repeat(Hv)
    ori = _answer_sums(eng.answer_logits(hf, ans, round_logits).view(1, n))[0] if qc.exact else None
    pos = {l: i for i, l in enumerate(layers)}
    for grp in sweep_groups(layers, sp.num_layers, SWEEP_GROUP):
        if len(grp) == 1:
            hvs = {grp[0]: layer_variants(eng, qc, grp[0], cb.bias, cb.W, n, p0=p0)}      # [Hv, n, D]
        else:
            hvs = group_variants(eng, qc, grp, cb.bias, cb.W, n, p0=p0)
        for l, hv in hvs.items():
            sums = _answer_sums(eng.answer_logits(hv.reshape(-1, sp.hidden), ans_rep, round_logits).view(Hv, n))
            out[pos[l]] = ori - sums if qc.exact else sums[0] - sums[1:]   # ori - cur
    return out


def _flop_parts(spec):
    """Per-row GEMM flops of one decoder layer by part: (q, k | v, o_proj + MLP), and the attention count."""
    D, F = spec.hidden, spec.intermediate
    fq = 2.0 * D * spec.q_size
    fkv = 2.0 * D * 2 * spec.kv_size
    frest = 2.0 * (spec.q_size * D + 3 * D * F)

    def attn(tq, s):   # tq queries at positions s-tq .. s-1, causal: QK^T + PV over the visible keys
        vis = tq * (s - tq) + tq * (tq + 1) / 2.0
        return 4.0 * spec.head_dim * spec.num_heads * vis
    return fq, fkv, frest, attn


def sweep_flops(spec, T: int, n_ans: int, p0: int = 0, layers=None) -> float:
    """ALGORITHMIC GEMM + attention flops of ie_question(layers=...) -- the work the IE of SURVEY §8(d) needs, the
    step roofline's numerator: one baseline forward plus, per swept layer l, the all-heads-biased attention of
    layer l and H = num_heads variant batches (head h of layer l re-weighted) through o_proj + MLP of layer l and
    the layers above.  Rows before p0 (the first biased key) are equal in every variant and are not recomputed
    (prefix skip).  The last layer of every forward needs K / V of every row but q, attention, o_proj and MLP of the
    n answer rows only.  What the sweep executes beyond this (the un-perturbed 33rd variant of the default mode, the
    GEMMs' pad rows, the baseline's last-layer q over every row) is sweep_flops_executed()."""
    L, H = spec.num_layers, spec.num_heads
    fq, fkv, frest, attn = _flop_parts(spec)
    p0 = max(0, min(p0, T - n_ans))
    Ts = T - p0
    lay = fq + fkv + frest
    last_layer = lambda t: fkv * t + (fq + frest) * n_ans + attn(n_ans, t)   # K/V of every row, the rest on n rows
    # baseline: L-1 full layers + the last layer
    f = (L - 1) * (lay * T + attn(T, T)) + last_layer(T)
    for l in (range(L) if layers is None else layers):
        rows = n_ans if l == L - 1 else Ts
        f += attn(rows, T)                                              # all-heads-biased attention of layer l
        f += H * frest * rows                                           # o_proj + MLP of layer l, H variants
        for l2 in range(l + 1, L):
            f += H * (fkv * Ts + (fq + frest) * n_ans + attn(n_ans, T) if l2 == L - 1
                      else lay * Ts + attn(Ts, T))
    return f


def sweep_flops_executed(spec, T: int, n_ans: int, p0: int = 0, layers=None, base_variant: bool = True,
                         group: int = 1) -> float:
    """The GEMM + attention flops ie_question EXECUTES: sweep_flops plus the un-perturbed variant each batch carries
    (base_variant: the mode without row-exactness), the pad rows of the suffix layers' GEMMs (engine.padded_rows: the
    256-row macro tile, then the measured row table) with the batches grouped as sweep_groups(.., group) groups them,
    and the baseline forward's last-layer q over every row."""
    from .engine import padded_rows
    L, H = spec.num_layers, spec.num_heads
    Hv = H + 1 if base_variant else H
    fq, fkv, frest, attn = _flop_parts(spec)
    p0 = max(0, min(p0, T - n_ans))
    Ts = T - p0
    lay = fq + fkv + frest
    f = (L - 1) * (lay * T + attn(T, T)) + (fq + fkv) * T + frest * n_ans + attn(n_ans, T)
    for grp in sweep_groups(range(L) if layers is None else layers, L, group):
        if grp == [L - 1]:                                              # the last layer: answer rows only
            f += attn(n_ans, T) + frest * Hv * n_ans
            continue
        nseq = 0
        m_prev = 0                                                      # padded rows of the running batch
        for l2 in range(grp[0], L):
            joins = l2 in grp
            if joins:
                f += attn(Ts, T)                                        # the joining layer's biased attention
            if nseq:                                                    # the running sequences' own layer l2
                if l2 == L - 1:
                    f += fkv * m_prev + (fq + frest) * nseq * n_ans + nseq * attn(n_ans, T)
                    continue
                f += (fq + fkv) * m_prev + nseq * attn(Ts, T)
            nseq += Hv if joins else 0
            m_prev = padded_rows(nseq * Ts, spec, no_tail=not base_variant)
            f += frest * m_prev                                         # o_proj + MLP over every row of the batch
    return f
