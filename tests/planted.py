"""Planted-IE model: random-init Llama-architecture weights in which a designed set of heads has a large,
sign-controlled, well separated indirect effect, so that the top-k head ranking of find_best_heads.py:113-150 has
boundary gaps far above bf16 noise at chosen k.  Test infrastructure only.

Why: with plain random weights the IE of re_weighting.py:152-175 (sum of the answer-token logits without the hook
minus the same sum with the fake passage masked for one head) is ~0.01 per head while every bf16 implementation —
the reference's own included — is ~0.1 off the float32 truth, so "identical top-k set" cannot be decided.  Here the
signal of the planted heads is 10-100x that noise and the rest of the network stays random.

Mechanism (D residual dims, head_dim d, RoPE pairs (i, i + d/2)):
  * private residual dims: BF (set only in the BOS token's embedding), CST (a constant in every token's embedding)
    and one channel CH_i per planted pair.  No random weight reads or writes them: their columns are zeroed in
    every q/k/v and gate/up weight and their rows in every o_proj / down weight.  lm_head reads every CH_i with the
    same weight -c0 for all vocabulary rows.
  * a planted kv group g of layer l: key dim s = d/2 - 1 (RoPE frequency ~1e-6: no rotation over a prompt) reads
    only BF, so only the BOS keys have k_s != 0 (an attention sink); the query dim s of its q-heads reads only CST,
    so every query row scores the BOS keys high; value dim 0 reads only BF, so v_0 = 1 at BOS and exactly 0 at every
    other key.  A head's value-dim-0 output is then its attention mass on BOS, p_B.
  * pairs (h+, h-) of q-heads of the group carry identical q weights (identical attention).  o_proj maps value dim
    0 of h+ to CH_i with +s_i and of h- with -s_i and nothing else of either head, so in the un-hooked forward
    CH_i = s_i (p_B - p_B) = 0 exactly and the baseline network does not depend on any planted parameter.
  * masking the fake passage for h+ (the sweep's scores [0,1,1,1,1] make it -inf) moves its mass onto the rest,
    p_B' = p_B / (1 - p_F) > p_B, so CH_i rises by s_i (p_B' - p_B), every answer logit falls by
    c0 * w_norm * dCH / rms, and IE(h+) > 0; IE(h-) is the same with the opposite sign.  To first order (CH_i is 0
    at baseline, so the final RMSNorm's scale moves only at second order) IE(h+) = s_i * u_i with
    u_i = c0 * sum_r w_norm[CH_i] (p_B' - p_B)_r / rms_r over the answer rows r; calibrate() measures u_i on the
    float32 network and sets s_i = target_i / mean_q u_i.
Ranking layout with P pairs in H_tot heads: ranks 1..P are the planted h+ in tiers of targets, P+1..H_tot-P the
random heads (|IE| ~ 0.01-0.1), the last P the planted h-.  Designed boundaries: the tier edges, P and H_tot - P
(with P = 130 on Llama-3-8B: 1024 - 130 = 894, the k of datasets/nq/llama3/selected_heads.json).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

import numpy as np
import torch

# Llama-3-8B default: 130 pairs in tiers (count, largest target, smallest target) -> boundaries 10, 50, 100, 130, 894.
# Round 4: every designed boundary gap >= 1.8 (round 3: 0.99 at k = 100, 1.26 / 1.34 at 130 / 894
# against a 3 x noise bar of 1.13), i.e. >= 1.5 x the bar at round 3's noise: tier edges 10.5 | 8.5, 7.0 | 5.0,
# 4.5 | 2.6, and the last tier's 2.3 against random heads of |IE| <= 0.34; the top target drops 16 -> 12, which also
# shrinks the bf16 noise of the largest IEs.
TIERS_LLAMA3 = ((10, 12.0, 10.5), (40, 8.5, 7.0), (50, 5.0, 4.5), (30, 2.6, 2.3))


@dataclass
class PlantLayout:
    bf: int
    cst: int
    channels: List[int]
    pairs: List[Tuple[int, int, int, int]]           # (layer, kv group, h+, h-), index = channel index
    targets: np.ndarray                              # IE target of pair i's h+ (h- gets -target)
    boundaries: List[int]                            # designed top-k boundaries
    bos_id: int
    c0: float
    sink_dim: int
    beta: List[float] = field(default_factory=list)  # per-pair query sink strength
    scales: np.ndarray = None                        # s_i after calibrate()

    def positive(self):
        return [(l, hp) for l, _, hp, _ in self.pairs]

    def negative(self):
        return [(l, hm) for l, _, _, hm in self.pairs]


def _tier_targets(tiers) -> Tuple[np.ndarray, List[int]]:
    vals, bounds, n = [], [], 0
    for cnt, hi, lo in tiers:
        vals.extend(np.linspace(hi, lo, cnt).tolist() if cnt > 1 else [hi])
        n += cnt
        bounds.append(n)
    return np.asarray(vals, dtype=np.float64), bounds


def plant_structure(eng, tiers=TIERS_LLAMA3, seed: int = 7, bos_id: int = 0, c0: float = 8.0,
                    bos_flag: float = 8.0, const: float = 1.0, q_random_scale: float = 0.25) -> PlantLayout:
    """Rewrite the engine's random weights in place (structure only: sink / value / scale parameters are set by
    calibrate()).  Returns the layout."""
    sp = eng.spec
    L, D, Hq, Hkv, d = sp.num_layers, sp.hidden, sp.num_heads, sp.num_kv_heads, sp.head_dim
    G = Hq // Hkv
    if G < 2 or d < 4:
        raise ValueError("planting needs >= 2 q-heads per kv head")
    targets, bounds = _tier_targets(tiers)
    P = len(targets)
    ppg = G // 2                                        # pairs per planted kv group
    n_groups = -(-P // ppg)
    # (layer, group) candidates: every layer once per round, rounds over kv groups, so the planted heads spread over
    # all depths before any layer gets a third group
    rounds = [(r * 3) % Hkv for r in range(Hkv)] if Hkv % 3 else list(range(Hkv))
    cands = [(l, (l * 3 + r) % Hkv) for r in rounds for l in range(L)]
    seen, groups = set(), []
    for c in cands:
        if c not in seen:
            seen.add(c)
            groups.append(c)
        if len(groups) == n_groups:
            break
    if len(groups) < n_groups:
        raise ValueError("too many pairs for this architecture")
    pairs = []
    for l, g in groups:
        for i in range(ppg):
            if len(pairs) < P:
                pairs.append((l, g, g * G + 2 * i, g * G + 2 * i + 1))
    rng = np.random.default_rng(seed)
    pairs = [pairs[i] for i in rng.permutation(P)]       # tiers spread over layers
    bf, cst = D - 1, D - 2
    channels = [D - 3 - i for i in range(P)]
    priv = torch.tensor([bf, cst] + channels, device=eng.device)
    q, kv = sp.q_size, sp.kv_size
    s = d // 2 - 1
    with torch.no_grad():
        for lw in eng.layers:
            lw.wqkv[:, priv] = 0
            lw.wgu[:, priv] = 0
            lw.wo[priv, :] = 0
            lw.wd[priv, :] = 0
        eng.embed[:, priv] = 0
        eng.embed[:, cst] = const
        eng.embed[bos_id, bf] = bos_flag
        eng.lm_head[:, priv] = 0
        eng.lm_head[:, channels] = -c0
        for l, g in groups:
            lw = eng.layers[l]
            for hh in range(g * G, (g + 1) * G):
                lw.wqkv[hh * d:(hh + 1) * d] *= q_random_scale
                lw.wqkv[hh * d + s] = 0
                lw.wqkv[hh * d + s + d // 2] = 0
                lw.wo[:, hh * d:(hh + 1) * d] = 0
            for r in (s, s + d // 2):
                lw.wqkv[q + g * d + r] = 0
            lw.wqkv[q + kv + g * d] = 0
            for i in range(ppg):                                     # identical q weights inside each pair
                hp, hm = g * G + 2 * i, g * G + 2 * i + 1
                lw.wqkv[hm * d:(hm + 1) * d] = lw.wqkv[hp * d:(hp + 1) * d]
    beta = [1.0 if i % 2 == 0 else 0.8 for i in range(P)]
    return PlantLayout(bf, cst, channels, pairs, targets, bounds + [Hq * L - P], bos_id, c0, s, beta)


class _LazyFp32:
    """The float32 network of tests/fp32_llama.py with each layer's weights upcast on use (no 4-byte copy of
    the whole model)."""

    def __init__(self, eng):
        from tests.fp32_llama import Fp32Llama
        self.eng = eng
        self.f = Fp32Llama.__new__(Fp32Llama)
        f = self.f
        f.sp = eng.spec
        f.embed = eng.embed
        f.norm = eng.norm.float()
        f.lm_head = eng.lm_head
        f.inv_freq = eng.inv_freq.float()
        f.attn_scaling = eng.attn_scaling
        up = lambda t: None if t is None else t.float()

        class _Layers:
            def __getitem__(_, l):
                lw = eng.layers[l]
                return dict(ln1=up(lw.ln1), wqkv=up(lw.wqkv), bqkv=up(lw.bqkv), wo=up(lw.wo), ln2=up(lw.ln2),
                            wgu=up(lw.wgu), wd=up(lw.wd))
        f.layers = _Layers()

    @torch.no_grad()
    def run(self, ids):
        """Per-layer inputs [L][T, D] and the final pre-norm residual [T, D] (float32)."""
        f = self.f
        T = ids.numel()
        cos, sin = f.rope(T, f.norm.device)
        mask = f.causal(T, f.norm.device).expand(f.sp.num_heads, T, T)
        h = f.embed[ids.view(-1)].float()
        hs = []
        for l in range(f.sp.num_layers):
            hs.append(h)
            h = f.layer(h, l, cos, sin, mask)
        return hs, h, cos, sin


def _rms(x, eps):
    return torch.sqrt(x.pow(2).mean(-1) + eps)


@torch.no_grad()
def calibrate(eng, lay: PlantLayout, questions: Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]],
              sink_score: float = 5.3, k_sink: float = 7.7) -> dict:
    """Set the sink / value weights per layer from the measured residual scale, then s_i = target_i / mean_q u_i.

    questions: (ids [T], w16 [W] fp16 credibility weights, answer ids [n]) as the sweep receives them."""
    sp = eng.spec
    d, G = sp.head_dim, sp.num_heads // sp.num_kv_heads
    q, kv = sp.q_size, sp.kv_size
    s = lay.sink_dim
    net = _LazyFp32(eng)
    # 1. residual scale at every layer input: BOS row (position 0) and the median over the other rows of question 0
    ids0 = questions[0][0]
    hs, _, _, _ = net.run(ids0)
    rms_bos = [float(_rms(h[0], sp.eps)) for h in hs]
    rms_tok = [float(_rms(h[1:], sp.eps).median()) for h in hs]
    q_sink = sink_score * d ** 0.5 / k_sink
    with torch.no_grad():
        for l, g in sorted({(l, g) for l, g, _, _ in lay.pairs}):
            lw = eng.layers[l]
            bfn = float(lw.ln1[lay.bf]) * float(eng.embed[lay.bos_id, lay.bf]) / rms_bos[l]
            cstn = float(lw.ln1[lay.cst]) * float(eng.embed[lay.bos_id, lay.cst]) / rms_tok[l]
            lw.wqkv[q + g * d + s, lay.bf] = k_sink / bfn                 # k_s(BOS) = k_sink
            lw.wqkv[q + kv + g * d, lay.bf] = 1.0 / bfn                   # v_0(BOS) = 1, 0 elsewhere
            for i, (l2, g2, hp, hm) in enumerate(lay.pairs):
                if (l2, g2) == (l, g):
                    for hh in (hp, hm):
                        lw.wqkv[hh * d + s, lay.cst] = lay.beta[i] * q_sink / cstn
    # 2. u_i on the float32 network: first-order IE of pair i's h+ per unit o_proj scale
    P = len(lay.pairs)
    u = np.zeros((len(questions), P))
    pb = np.zeros((len(questions), P))
    for qi, (ids, w16, ans) in enumerate(questions):
        hs, hfin, cos, sin = net.run(ids)
        T, n = ids.numel(), ans.numel()
        rows = torch.arange(T - n, T, device=ids.device)
        inv_rms = 1.0 / _rms(hfin[rows], sp.eps)                           # [n]
        bias = torch.zeros(T, device=ids.device)
        W = w16.numel()
        bias[:W] = torch.log(w16.to(ids.device).float())
        causal = torch.arange(T, device=ids.device)[None, :] <= rows[:, None]   # [n, T]
        for i, (l, g, hp, _) in enumerate(lay.pairs):
            wl = net.f.layers[l]
            x = net.f.rms(hs[l], wl["ln1"])
            qh = net.f.rot((x[rows] @ wl["wqkv"][hp * d:(hp + 1) * d].t()), cos[rows], sin[rows])
            kh = net.f.rot(x @ wl["wqkv"][q + g * d:q + (g + 1) * d].t(), cos, sin)
            v0 = x @ wl["wqkv"][q + kv + g * d]
            sc = (qh @ kh.t()) * d ** -0.5
            sc = sc.masked_fill(~causal, float("-inf"))
            o = torch.softmax(sc, -1) @ v0
            o2 = torch.softmax(sc + bias[None], -1) @ v0
            wn = float(eng.norm[lay.channels[i]].float())
            u[qi, i] = float((lay.c0 * wn * (o2 - o) * inv_rms).sum())
            pb[qi, i] = float(torch.softmax(sc, -1)[:, :2].sum(-1).mean())
    ubar = u.mean(0)
    if (ubar <= 0).any():
        raise RuntimeError(f"planted heads without a positive first-order IE: {np.nonzero(ubar <= 0)[0].tolist()}")
    lay.scales = lay.targets / ubar
    with torch.no_grad():
        for i, (l, g, hp, hm) in enumerate(lay.pairs):
            wo = eng.layers[l].wo
            wo[lay.channels[i], hp * d] = float(lay.scales[i])
            wo[lay.channels[i], hm * d] = -float(lay.scales[i])
    return {"u": u, "p_bos": pb, "rms_bos": rms_bos, "rms_tok": rms_tok}


def designed_ranking(lay: PlantLayout, num_layers: int, num_heads: int):
    """(top set per designed boundary k) from the layout alone: the first P boundaries are prefixes of the planted
    h+ in target order; k = H_tot - P is everything but the planted h-."""
    order = np.argsort(-lay.targets, kind="stable")
    pos = lay.positive()
    out = {}
    for k in lay.boundaries:
        if k <= len(pos):
            out[k] = {pos[i] for i in order[:k]}
        else:
            neg = set(lay.negative())
            out[k] = {(l, h) for l in range(num_layers) for h in range(num_heads)} - neg
    return out
