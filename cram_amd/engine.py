"""CrAMEngine: Llama-3 / Qwen2-family forward on MI355X built around the HIP attention kernels.

The reference runs the model through transformers with a dense-mask hook
(re_weighting.py:116-138 generate path, :152-175 IE path).  The engine runs the
same network (weights taken from a transformers model, or random-init of the
same shapes for throughput runs) with:
  * fused QKV and gate/up projections (one hipBLASLt GEMM each, via torch),
  * credibility-biased attention from libcram_attn (prefill MFMA kernel,
    decode split-S kernel) reading q/k/v straight out of the QKV buffer,
  * a static per-batch KV cache ([L][B][Hkv][S_max][d], model dtype) and a decode
    step whose attention reads per-row lengths from device memory, so a whole
    greedy step can be captured in one hipGraph and replayed,
  * answer-token logits by the fp32 gather kernel instead of the full-vocab
    lm_head (IE sweep).
Elementwise ops follow transformers' exact op order and rounding points
(LlamaRMSNorm, apply_rotary_pos_emb, LlamaMLP) so the engine tracks the
reference numerics; only GEMM reduction order and the attention kernel differ.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from . import gemm_tune, ops
from .bias import CredibilityBias


@dataclass
class ModelSpec:
    num_layers: int
    hidden: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate: int
    vocab: int
    eps: float
    qkv_bias: bool
    family: str = "llama"

    @property
    def q_size(self):
        return self.num_heads * self.head_dim

    @property
    def kv_size(self):
        return self.num_kv_heads * self.head_dim

    @staticmethod
    def from_config(cfg) -> "ModelSpec":
        hd = getattr(cfg, "head_dim", None) or cfg.hidden_size // cfg.num_attention_heads
        fam = "qwen2" if cfg.model_type.startswith("qwen2") else "llama"
        return ModelSpec(cfg.num_hidden_layers, cfg.hidden_size, cfg.num_attention_heads,
                         getattr(cfg, "num_key_value_heads", cfg.num_attention_heads), hd, cfg.intermediate_size,
                         cfg.vocab_size, cfg.rms_norm_eps, fam == "qwen2" or bool(getattr(cfg, "attention_bias", False)),
                         fam)

    # the shapes BASELINE.json names
    @staticmethod
    def llama3_8b() -> "ModelSpec":
        return ModelSpec(32, 4096, 32, 8, 128, 14336, 128256, 1e-5, False, "llama")

    @staticmethod
    def qwen2_7b() -> "ModelSpec":
        return ModelSpec(28, 3584, 28, 4, 128, 18944, 152064, 1e-6, True, "qwen2")

    # the reference's default model (re_weighting.py:22 model_name="Llama-2-13b-chat-hf"): MHA, fp16 checkpoint
    @staticmethod
    def llama2_13b() -> "ModelSpec":
        return ModelSpec(40, 5120, 40, 40, 128, 13824, 32000, 1e-5, False, "llama")

    def layer_flops(self, T: int) -> float:
        """GEMM flops of one decoder layer over T tokens (2 * params * T)."""
        p = self.hidden * (self.q_size + 2 * self.kv_size) + self.q_size * self.hidden + 3 * self.hidden * self.intermediate
        return 2.0 * p * T


ROW_ALIGN = 256
# gate/up + SiLU-mul on cram_gemm's fused epilogue (CrAMEngine.mlp); CRAM_FUSED_MLP=0: hipBLASLt + cram_silu_mul (A/B)
FUSED_MLP = os.environ.get("CRAM_FUSED_MLP", "1") != "0"
# o_proj / down_proj with the residual add in cram_gemm's epilogue (CrAMEngine.o_proj_norm / mlp_residual) at the same
# row counts; CRAM_FUSED_RESIDUAL=0: the add inside the next RMSNorm instead (A/B)
FUSED_RESIDUAL = os.environ.get("CRAM_FUSED_RESIDUAL", "1") != "0"
# q/k/v projection (+ bias) with RoPE in cram_gemm's epilogue (head_dim 128) at the same row counts;
# CRAM_FUSED_QKV=0: hipBLASLt + cram_rope_inplace / cram_rope_split (A/B)
FUSED_QKV = os.environ.get("CRAM_FUSED_QKV", "1") != "0"
# the sparse last wave of the residual GEMMs' tiles through split-K (CrAMEngine._gemm_residual); 0 = one launch (A/B)
TAIL_SPLIT = os.environ.get("CRAM_TAIL_SPLIT", "1") != "0"
# packed-prefill chunk bound (tokens): the IE sweep's GEMM row count, where the GEMMs already run at full rate;
# config 2 measured 75.75-75.94 q/s at 32k, 75.84 at 64k, 75.37 at 16k (r04, profiles/r04/ab_prefill_chunk/);
# CRAM_PREFILL_CHUNK_ROWS overrides it (A/B)
PREFILL_CHUNK_ROWS = int(os.environ.get("CRAM_PREFILL_CHUNK_ROWS", "32768"))
# the sweep's last suffix layer projects q for the answer rows only (layer_rows, out_rows + prefix);
# CRAM_LAST_Q_ROWS=0 projects every row's q as the other layers do (A/B)
LAST_Q_ROWS_ONLY = os.environ.get("CRAM_LAST_Q_ROWS", "1") != "0"
# The prompts of one decode batch open with the same tokens (the chat template's system turn and the instruction line:
# 37 of the ~906 tokens of a Llama-3 NQ prompt): their K/V are computed once, copied into every cache row, and the
# packed prefill runs the suffixes only, attending over the cache (cram_attn_prefill_varlen_cached).
# CRAM_PREFIX_SHARE=0 prefills whole prompts (A/B, tests).
PREFIX_SHARE = os.environ.get("CRAM_PREFIX_SHARE", "1") != "0"
PREFIX_SHARE_MIN_ROWS = 16
# ... and the decode attention reads those rows from cache row 0 (cram_attn_decode_shared: one HBM stream of the
# opening per step instead of one per row, bit-identical); CRAM_SHARED_DECODE_READ=0 reads every row's copy (A/B)
SHARED_DECODE_READ = os.environ.get("CRAM_SHARED_DECODE_READ", "1") != "0"


def padded_rows(M: int, spec: Optional["ModelSpec"] = None, no_tail: bool = False) -> int:
    """GEMM row count for M rows: rounded up to the 256-row macro tile and, for the Llama-3-8B projection shapes, to
    the row count within +2048 that minimises the measured per-layer GEMM time plus the per-row non-GEMM work
    (data/gemm_rows.json, the engine's own fused GEMMs with the residual tail split: ~311-314 ns per row at most
    row counts, 307-309 at multiples of 4096; round 3's hipBLASLt table had 290 vs 305-315).  no_tail: the table of
    the same GEMMs without the split-K tail (the IE sweep's row-exact batches, 16k-131k rows: their grouped batches
    reach ~120k rows), where a row count whose N = 4096 tiles end in a sparse wave costs that whole wave."""
    Mp = -(-M // ROW_ALIGN) * ROW_ALIGN
    tab = _row_table(spec, no_tail)
    if tab is None or Mp not in tab:
        return Mp
    # within +2048 rows, or +1/16 of M for the grouped sweep batches (~60-120k rows)
    cands = [m for m in range(Mp, Mp + max(2048, Mp // 16) + 1, ROW_ALIGN) if m in tab]
    return min(cands, key=lambda m: (tab[m] + ROW_COST_MS * m, m))


# non-GEMM work per GEMM row of a suffix layer (attention, RMSNorm, copies: ~5.7 % of the sweep step against the fused
# GEMMs' 94 % in round 4's rocprof summary, i.e. ~19 ns per row next to ~311 ns of GEMM)
ROW_COST_MS = 19e-6
_ROW_TABLES = {}


def _row_table(spec, no_tail: bool = False) -> Optional[dict]:
    if spec is None or os.environ.get("CRAM_ROW_TABLE", "1") == "0":    # A/B switch: plain 256-row rounding
        return None
    key = (spec.hidden, spec.intermediate, spec.q_size + 2 * spec.kv_size, no_tail)
    if key not in _ROW_TABLES:
        import json
        fn = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "gemm_rows.json")
        tab = None
        try:
            with open(fn) as f:
                d = json.load(f)
            shp = d["shape"]
            name = "layer_gemm_ms_no_tail" if no_tail else "layer_gemm_ms"
            if key[:3] == (shp["hidden"], shp["intermediate"], shp["qkv"]) and name in d:
                tab = {int(m): float(t) for m, t in d[name].items()}
        except (OSError, ValueError, KeyError):
            tab = None
        _ROW_TABLES[key] = tab
    return _ROW_TABLES[key]


def configure_blas(lib: str = "hipblas") -> None:
    """Select torch's default GEMM backend.  hipBLASLt and rocBLAS measure equal per Llama-3-8B layer at the sweep's
    row counts (tools/gemm_bench.py; an earlier 13 % QKV gap was a cold-clock ordering artefact) and in the full
    bench; the shapes where the default pick is slow are pinned by gemm_tune."""
    torch.backends.cuda.preferred_blas_library(lib)


class LayerW:
    __slots__ = ("ln1", "wqkv", "bqkv", "wo", "ln2", "wgu", "wd", "wgu_il", "wgu_il_key", "wgu_tail", "wgu_tail_key")


class CrAMEngine:
    def __init__(self, spec: ModelSpec, layers: List[LayerW], embed: torch.Tensor, norm: torch.Tensor,
                 lm_head: torch.Tensor, inv_freq: torch.Tensor, attn_scaling: float = 1.0):
        self.spec = spec
        self.layers = layers
        self.embed = embed
        self.norm = norm
        self.lm_head = lm_head
        self.inv_freq = inv_freq.float()
        self.attn_scaling = float(attn_scaling)
        self.device = embed.device
        self.dtype = embed.dtype
        self.scale = spec.head_dim ** -0.5
        # the IE sweep's row-exact modes (sweep.py): fused_any_rows puts every projection on the 4-wave kernel
        # whatever the row count; no_tail_split (the baseline forward) keeps every row of a launch on it too, so a
        # row computes the same bits there as in the whole waves of any variant batch
        self.fused_any_rows = False
        self.no_tail_split = False
        if self.device.type == "cuda":
            gemm_tune.ensure()          # pinned q/k/v and o_proj GEMM solutions, used inside gemm_tune.pinned()

    # ------------------------------------------------------------------ construction
    SUPPORTED = ("llama", "qwen2")

    @staticmethod
    def supports(model) -> bool:
        """The engine re-implements the Llama / Qwen2 decoder (RMSNorm, RoPE, SwiGLU, GQA)."""
        return getattr(model.config, "model_type", "") in CrAMEngine.SUPPORTED

    @staticmethod
    def from_hf(model) -> "CrAMEngine":
        """Share the transformers model's weights (q/k/v and gate/up are concatenated once)."""
        spec = ModelSpec.from_config(model.config)
        base = model.model
        layers = []
        for blk in base.layers:
            a, m = blk.self_attn, blk.mlp
            lw = LayerW()
            lw.ln1 = blk.input_layernorm.weight.data
            lw.wqkv = torch.cat([a.q_proj.weight.data, a.k_proj.weight.data, a.v_proj.weight.data], 0).contiguous()
            lw.bqkv = (torch.cat([a.q_proj.bias.data, a.k_proj.bias.data, a.v_proj.bias.data], 0).contiguous()
                       if a.q_proj.bias is not None else None)
            lw.wo = a.o_proj.weight.data
            lw.ln2 = blk.post_attention_layernorm.weight.data
            lw.wgu = torch.cat([m.gate_proj.weight.data, m.up_proj.weight.data], 0).contiguous()
            lw.wd = m.down_proj.weight.data
            layers.append(lw)
        rot = base.rotary_emb
        return CrAMEngine(spec, layers, base.embed_tokens.weight.data, base.norm.weight.data,
                          model.lm_head.weight.data, rot.inv_freq.detach().to(model.device),
                          getattr(rot, "attention_scaling", 1.0))

    @staticmethod
    def random(spec: ModelSpec, device, seed: int = 0, std: float = 0.02, rope_theta: float = 500000.0,
               dtype=torch.bfloat16) -> "CrAMEngine":
        """Random-init weights of the given architecture (throughput runs; no checkpoint offline)."""
        g = torch.Generator(device=device).manual_seed(seed)

        def rnd(*shape, s=std):
            return (torch.randn(*shape, generator=g, device=device, dtype=torch.float32) * s).to(dtype)

        def ones_ish(n):
            return (1.0 + 0.05 * torch.randn(n, generator=g, device=device)).to(dtype)

        layers = []
        for _ in range(spec.num_layers):
            lw = LayerW()
            lw.ln1 = ones_ish(spec.hidden)
            lw.wqkv = rnd(spec.q_size + 2 * spec.kv_size, spec.hidden)
            lw.bqkv = rnd(spec.q_size + 2 * spec.kv_size) if spec.qkv_bias else None
            lw.wo = rnd(spec.hidden, spec.q_size)
            lw.ln2 = ones_ish(spec.hidden)
            lw.wgu = rnd(2 * spec.intermediate, spec.hidden)
            lw.wd = rnd(spec.hidden, spec.intermediate)
            layers.append(lw)
        embed = rnd(spec.vocab, spec.hidden, s=1.0)
        lm_head = rnd(spec.vocab, spec.hidden)
        inv_freq = 1.0 / (rope_theta ** (torch.arange(0, spec.head_dim, 2, dtype=torch.float32, device=device)
                                         / spec.head_dim))
        return CrAMEngine(spec, layers, embed, ones_ish(spec.hidden), lm_head, inv_freq)

    # ------------------------------------------------------------------ elementwise (fused HIP kernels)
    def rmsnorm(self, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        """LlamaRMSNorm (cram_rmsnorm)."""
        return ops.rmsnorm(x if x.is_contiguous() else x.contiguous(), w, self.spec.eps)

    def add_rmsnorm(self, delta: torch.Tensor, h: torch.Tensor, w: torch.Tensor):
        """(h + delta, LlamaRMSNorm(h + delta)) in one pass."""
        return ops.rmsnorm(delta, w, self.spec.eps, residual=h if h.is_contiguous() else h.contiguous())

    def rope_tables(self, P: int):
        """cos, sin (model dtype) [P, d] for positions 0..P-1 (LlamaRotaryEmbedding.forward arithmetic)."""
        freqs = torch.arange(P, device=self.device, dtype=torch.float32)[:, None] * self.inv_freq[None, :]
        emb = torch.cat((freqs, freqs), dim=-1)
        return (emb.cos() * self.attn_scaling).to(self.dtype), (emb.sin() * self.attn_scaling).to(self.dtype)

    def mlp(self, x: torch.Tensor, lw: LayerW) -> torch.Tensor:
        """LlamaMLP: down(rnd(silu(gate)) * up).  Row counts of the sweep and the packed prefill run gate/up on
        cram_gemm's 4-wave kernel with the SiLU-mul in its epilogue (the [M, 2F] projection never reaches HBM;
        1.05x hipBLASLt + cram_silu_mul at M = 29k, tools/gemm_ab_knob.py), same rounding points as the pair."""
        F = self.spec.intermediate
        if self._fused_mlp_ok(x):
            act = ops.gemm(x, self._gate_up_interleaved(lw), ops.GEMM_SILU_MUL)
        else:
            act = ops.silu_mul(ops.linear(x, lw.wgu), F)
        return ops.linear(act, lw.wd)

    def o_proj_norm(self, a: torch.Tensor, lw: LayerW, h: torch.Tensor):
        """(h + o_proj(a), RMSNorm_ln2 of it) over row buffers a [M, q_size], h [M, D].  At the fused kernels' row
        counts the residual add runs in o_proj's epilogue (cram_gemm_residual) and the norm reads one tensor;
        otherwise o_proj is F.linear and the add runs inside the norm.  Same rounding points either way."""
        if self._fused_residual_ok(a):
            h2 = self._gemm_residual(a, lw.wo, h)
            return h2, ops.rmsnorm(h2, lw.ln2, self.spec.eps)
        return ops.rmsnorm(ops.linear(a, lw.wo), lw.ln2, self.spec.eps, residual=h)

    def mlp_residual(self, x: torch.Tensor, lw: LayerW, h: torch.Tensor):
        """The MLP half of a decoder layer over row buffers x, h [M, D]: (h + mlp(x), None) with the add in
        down_proj's epilogue at the fused kernels' row counts, else (h, mlp(x)) -- the add left pending for the next
        consumer's RMSNorm (its residual input)."""
        if self._fused_residual_ok(x):
            act = ops.gemm(x, self._gate_up_interleaved(lw), ops.GEMM_SILU_MUL)
            return self._gemm_residual(act, lw.wd, h), None
        return h, self.mlp(x, lw)

    # the fused GEMMs from one full 256-row tile: every sweep / packed-prefill call, and the sweep's baseline forward
    # (T ~ 1k rows, 0.2 % of the sweep's FLOPs) so no separate RoPE / SiLU-mul pass is left in the sweep
    FUSED_MLP_MIN_ROWS = 256

    def _fused_mlp_ok(self, x: torch.Tensor) -> bool:
        if not FUSED_MLP or self.device.type != "cuda" or self.dtype not in (torch.bfloat16, torch.float16):
            return False
        D, F = self.spec.hidden, self.spec.intermediate
        M = x.numel() // x.shape[-1]
        return ((M >= self.FUSED_MLP_MIN_ROWS or self.fused_any_rows) and (2 * F) % 256 == 0 and D % 64 == 0
                and D >= 128)

    def _gemm_residual(self, x: torch.Tensor, w: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
        """h + x @ w^T on row buffers with the add in the GEMM epilogue.  The 4-wave kernel runs one 256 x 256 tile
        per CU, so a launch takes ceil(tiles / CUs) tile times: at the sweep's row counts the N = 4096 projections'
        last wave is often a few tiles (M = 29,184: 1,824 tiles = 7 waves + 32), and o_proj / down_proj (down: 3.5x
        the K) then leave ~7/8 of the chip idle for a whole tile time.  Rows past the last whole wave go instead
        through the split-K form with the same epilogue, their K cut into ranges until the tail fills the chip."""
        M, K, N = x.numel() // x.shape[-1], x.shape[-1], w.shape[0]
        if self.no_tail_split:                 # one kernel for every row
            return ops.gemm(x, w, residual=h)
        ntn, mt = N // 256, -(-M // 256)
        waves = mt * ntn // self.num_cus
        mt_main = waves * self.num_cus // ntn
        tail = (mt - mt_main) * ntn
        if TAIL_SPLIT and waves >= 1 and 0 < tail <= self.num_cus // 2 and mt_main * 256 < M:
            splits = 1
            while (tail * splits * 2 <= self.num_cus and K % (64 * splits * 2) == 0
                   and K // (64 * splits * 2) >= 4):
                splits *= 2
            if splits > 1:
                Mm = mt_main * 256
                out = torch.empty_like(h)
                ops.gemm(x[:Mm], w, residual=h[:Mm], out=out[:Mm])
                ops.gemm_splitk(x[Mm:M], w, splits, residual=h[Mm:M], out=out[Mm:M])
                return out
        return ops.gemm(x, w, residual=h)

    @property
    def num_cus(self) -> int:
        if getattr(self, "_num_cus", None) is None:
            self._num_cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        return self._num_cus

    def _fused_qkv_ok(self, x: torch.Tensor, lw: LayerW) -> bool:
        sp = self.spec
        return (FUSED_QKV and self._fused_mlp_ok(x) and sp.head_dim == 128
                and (sp.num_heads + 2 * sp.num_kv_heads) % 2 == 0)

    def _fused_residual_ok(self, x: torch.Tensor) -> bool:
        sp = self.spec
        return (FUSED_RESIDUAL and self._fused_mlp_ok(x) and sp.hidden % 256 == 0 and sp.q_size % 64 == 0
                and sp.intermediate % 64 == 0)

    def _gate_up_interleaved(self, lw: LayerW) -> torch.Tensor:
        """lw.wgu with gate / up rows interleaved in blocks of 32 (cram_gemm's SiLU-mul layout), rebuilt whenever the
        checkpoint weight changes (tensor identity + torch's in-place version counter)."""
        w = lw.wgu
        key = (w.data_ptr(), w._version)
        if getattr(lw, "wgu_il_key", None) != key:
            lw.wgu_il = ops.interleave_gate_up(w, self.spec.intermediate).contiguous()
            lw.wgu_il_key = key
        return lw.wgu_il

    def _gate_up_tail(self, lw: LayerW, c0: int) -> torch.Tensor:
        """[gate[c0:]; up[c0:]] of lw.wgu (the split-K SiLU-mul layout) for the decode step's column tail, rebuilt
        whenever the checkpoint weight changes."""
        w, F = lw.wgu, self.spec.intermediate
        key = (w.data_ptr(), w._version, c0)
        if getattr(lw, "wgu_tail_key", None) != key:
            lw.wgu_tail = torch.cat([w[c0:F], w[F + c0:]]).contiguous()
            lw.wgu_tail_key = key
        return lw.wgu_tail

    def qkv(self, x: torch.Tensor, lw: LayerW, cos, sin, pos: Optional[torch.Tensor] = None):
        """x [B, T, D] -> roped q [B, T, Hq, d], k / v [B, T, Hkv, d]: strided views of one fused buffer."""
        sp = self.spec
        if self._fused_qkv_ok(x, lw) and x.is_contiguous():
            y = ops.gemm_rope(x, lw.wqkv, sp.num_heads, sp.num_kv_heads, sp.head_dim, cos, sin, T=x.shape[-2], pos=pos,
                              bias=lw.bqkv)
        else:
            y = ops.linear(x, lw.wqkv, lw.bqkv)
            ops.rope_inplace(y, sp.num_heads + sp.num_kv_heads, sp.head_dim, cos, sin, T=y.shape[-2], pos=pos)
        q = y[..., :sp.q_size].unflatten(-1, (sp.num_heads, sp.head_dim))
        k = y[..., sp.q_size:sp.q_size + sp.kv_size].unflatten(-1, (sp.num_kv_heads, sp.head_dim))
        v = y[..., sp.q_size + sp.kv_size:].unflatten(-1, (sp.num_kv_heads, sp.head_dim))
        return q, k, v

    # ------------------------------------------------------------------ prefill / full forward
    def attention(self, q, k, v, bias: Optional[torch.Tensor] = None, enable: Optional[torch.Tensor] = None,
                  W: int = 0) -> torch.Tensor:
        """q [B, Tq, Hq, d], k/v [B, S, Hkv, d] (token-major views) -> [B, Tq, Hq, d]."""
        return ops.attn_prefill(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale=self.scale,
                                bias=bias, enable=enable, W=W)

    def layer(self, h: torch.Tensor, l: int, cos, sin, bias=None, enable=None, W: int = 0,
              out_rows: Optional[int] = None) -> torch.Tensor:
        """One decoder layer over h [B, T, D].  out_rows=n computes attention/MLP for the last n rows only."""
        lw = self.layers[l]
        x = self.rmsnorm(h, lw.ln1)
        q, k, v = self.qkv(x, lw, cos, sin)
        if out_rows is not None:
            q = q[:, -out_rows:]
            h = h[:, -out_rows:]
        a = self.attention(q, k, v, bias, enable, W)
        h, x2 = self.add_rmsnorm(ops.linear(a.flatten(-2), lw.wo), h, lw.ln2)
        return h + self.mlp(x2, lw)

    def layer_rows(self, hbuf: torch.Tensor, B: int, T: int, l: int, cos, sin, bias=None, enable=None, W: int = 0,
                   out_rows: Optional[int] = None, delta: Optional[torch.Tensor] = None, prefix=None, join=None):
        """One decoder layer over a ROW buffer: rows [0, B*T) are B sequences of T tokens, rows beyond are
        alignment padding (GEMM M from padded_rows: the 256-row macro tile, then the measured row table; padding rows carry
        garbage and are never read back).  The layer input is hbuf [Mp, D], or hbuf + delta when the previous
        layer's MLP output is still pending (the residual add then runs inside this layer's first RMSNorm).
        Returns (h, mlp_out): the layer output is h + mlp_out, left for the next consumer to fuse (mlp_out None: h
        is the layer output, the add ran in down_proj's epilogue).
        out_rows=n returns [B*n, D] pairs (last n rows of every sequence).

        prefix=(k0, v0): the B sequences are SUFFIXES that start at position p0 = k0.shape[1] of a common
        prefix whose roped K/V at this layer are k0/v0 [1, p0, Hkv, d] (shared by all B sequences); row t of every
        suffix sits at position p0 + t (the only form: the fused path computes that position, the library path
        builds the same array).  Attention then runs over p0 + T keys per sequence.

        join=(a_new [M_new, q_size], h_new [M_new, D]): M_new more rows (whole sequences of T rows) enter here, after
        the attention, with their attention output given (the IE sweep's next perturbed layer, sweep.group_variants):
        o_proj + MLP run over the B * T rows and those in one launch each; the returned buffers hold B * T + M_new
        rows (padded as padded_rows picks)."""
        sp, lw = self.spec, self.layers[l]
        M = B * T
        if delta is None:
            x = ops.rmsnorm(hbuf, lw.ln1, sp.eps)
        else:
            hbuf, x = ops.rmsnorm(delta, lw.ln1, sp.eps, residual=hbuf)
        fused = self._fused_qkv_ok(x, lw)            # RoPE in the q/k/v GEMM's epilogue (cram_gemm_rope)
        if prefix is None:
            if fused:
                y = ops.gemm_rope(x, lw.wqkv, sp.num_heads, sp.num_kv_heads, sp.head_dim, cos, sin, T, rows=M,
                                  bias=lw.bqkv)
            else:
                y = ops.linear(x, lw.wqkv, lw.bqkv)
                ops.rope_inplace(y[:M], sp.num_heads + sp.num_kv_heads, sp.head_dim, cos, sin, T=T)
            y3 = y[:M].view(B, T, -1)
            k = y3[..., sp.q_size:sp.q_size + sp.kv_size].unflatten(-1, (sp.num_kv_heads, sp.head_dim))
            v = y3[..., sp.q_size + sp.kv_size:].unflatten(-1, (sp.num_kv_heads, sp.head_dim))
        else:                                        # [prefix | suffix] keys per sequence
            k0, v0 = prefix
            p0 = k0.shape[1]
            k = torch.empty((B, p0 + T, sp.num_kv_heads, sp.head_dim), dtype=self.dtype, device=self.device)
            v = torch.empty_like(k)
            k[:, :p0] = k0
            v[:, :p0] = v0
            # q roped in place; the suffix's roped k and its v land behind the prefix (no copy pass)
            if fused and out_rows is not None and LAST_Q_ROWS_ONLY:
                # the last layer reads q of the answer rows only: K / V of every row (the k | v rows of the fused
                # weight), q of the last out_rows rows of every sequence (a 1/3-size GEMM over 2/3 of the columns)
                n = out_rows
                qs = sp.q_size
                ops.gemm_rope(x, lw.wqkv[qs:], 0, sp.num_kv_heads, sp.head_dim, cos, sin, T, rows=M, kout=k, vout=v,
                              row0=p0, pos0=p0, bias=None if lw.bqkv is None else lw.bqkv[qs:])
                xa = x[:M].view(B, T, -1)[:, -n:].reshape(B * n, -1)
                yq = ops.gemm_rope(xa, lw.wqkv[:qs], sp.num_heads, 0, sp.head_dim, cos, sin, n,
                                   pos0=p0 + T - n, bias=None if lw.bqkv is None else lw.bqkv[:qs])
                q = yq.view(B, n, sp.num_heads, sp.head_dim)
                a = torch.empty((B * n, sp.q_size), dtype=self.dtype, device=self.device)
                ops.attn_prefill(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale=self.scale,
                                 bias=bias, enable=enable, W=W, out=a.view(B, n, sp.num_heads, sp.head_dim))
                hres = hbuf[:M].view(B, T, -1)[:, -n:].reshape(B * n, -1)
                h2, x2 = self.o_proj_norm(a, lw, hres)
                return self.mlp_residual(x2, lw, h2)
            if fused:
                # the suffix rows' positions are p0 + t: no position loads
                y = ops.gemm_rope(x, lw.wqkv, sp.num_heads, sp.num_kv_heads, sp.head_dim, cos, sin, T, rows=M,
                                  kout=k, vout=v, row0=p0, pos0=p0, bias=lw.bqkv)
            else:
                y = ops.linear(x, lw.wqkv, lw.bqkv)
                pos = (torch.arange(T, device=self.device, dtype=torch.int64) + p0).repeat(B)
                ops.rope_split(y[:M], sp.num_heads, sp.num_kv_heads, sp.head_dim, cos, sin, T, k, v, p0, pos=pos)
            y3 = y[:M].view(B, T, -1)
        q = y3[..., :sp.q_size].unflatten(-1, (sp.num_heads, sp.head_dim))
        if out_rows is None and join is not None:
            a_new, h_new = join
            Mt = M + a_new.shape[0]
            Mp = padded_rows(Mt, sp, no_tail=self.no_tail_split)
            a = torch.empty((Mp, sp.q_size), dtype=self.dtype, device=self.device)
            ops.attn_prefill(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale=self.scale, bias=bias,
                             enable=enable, W=W, out=a[:M].view(B, T, sp.num_heads, sp.head_dim))
            a[M:Mt] = a_new
            hres = torch.empty((Mp, sp.hidden), dtype=self.dtype, device=self.device)
            hres[:M] = hbuf[:M]
            hres[M:Mt] = h_new
        elif out_rows is None:
            a = torch.empty((hbuf.shape[0], sp.q_size), dtype=self.dtype, device=self.device)
            ops.attn_prefill(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale=self.scale, bias=bias,
                             enable=enable, W=W, out=a[:M].view(B, T, sp.num_heads, sp.head_dim))
            hres = hbuf
        else:
            n = out_rows
            a = torch.empty((B * n, sp.q_size), dtype=self.dtype, device=self.device)
            ops.attn_prefill(q[:, -n:].transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale=self.scale,
                             bias=bias, enable=enable, W=W, out=a.view(B, n, sp.num_heads, sp.head_dim))
            hres = hbuf[:M].view(B, T, -1)[:, -n:].reshape(B * n, -1)
        h2, x2 = self.o_proj_norm(a, lw, hres)
        return self.mlp_residual(x2, lw, h2)

    @torch.no_grad()
    def forward_hidden(self, ids: torch.Tensor, cb: Optional[CredibilityBias] = None,
                       out_rows: Optional[int] = None) -> torch.Tensor:
        """ids [B, T] -> final-norm hidden states [B, T or out_rows, D]."""
        B, T = ids.shape
        cos, sin = self.rope_tables(T)
        h = self.embed[ids]
        L = self.spec.num_layers
        for l in range(L):
            en = cb.enable[l] if cb is not None else None
            h = self.layer(h, l, cos, sin, cb.bias if cb is not None else None, en, cb.W if cb is not None else 0,
                           out_rows=out_rows if l == L - 1 else None)
        return self.rmsnorm(h, self.norm)

    @torch.no_grad()
    def logits(self, ids: torch.Tensor, cb: Optional[CredibilityBias] = None, last: Optional[int] = None):
        h = self.forward_hidden(ids, cb, out_rows=last)
        return ops.linear(h, self.lm_head)

    def answer_logits(self, hidden: torch.Tensor, ids: torch.Tensor, round_logits: bool = False) -> torch.Tensor:
        """hidden [n, D] (model dtype), ids int32 [n] -> fp32 [n] (HIP gather-dot)."""
        return ops.answer_logits(hidden.contiguous(), self.lm_head, ids, round_logits=round_logits)

    # ------------------------------------------------------------------ batched greedy decode
    @torch.no_grad()
    def generate(self, prompts: Sequence[torch.Tensor], weights16: Sequence[torch.Tensor], layers_to_heads: dict,
                 max_new_tokens: int = 100, eos_ids: Sequence[int] = (), bad_token_ids: Sequence[int] = (),
                 use_graph: bool = True, stop_on_eos: bool = True,
                 repetition_penalty: float = 1.0, phases: Optional[dict] = None,
                 bad_words_ids: Sequence[Sequence[int]] = ()) -> List[List[int]]:
        """Greedy decode of several prompts at once (per-row lengths, per-row credibility bias).

        Returns the generated ids of every prompt, truncated after its first EOS
        (tokens generated after EOS are never observed, so per-row results equal
        one-at-a-time generation as in re_weighting.py:127-132).  repetition_penalty != 1 applies transformers'
        RepetitionPenaltyLogitsProcessor (the checkpoint's generation_config, e.g. Qwen chat models ship 1.05)
        over each row's prompt and generated ids.
        bad_words_ids: transformers' NoBadWordsLogitsProcessor (generate(bad_words_ids=...), re_weighting.py:128-129):
        a one-id sequence is banned at every step, a longer one bans its last id whenever the row's ids so far (prompt
        + generated) end with its other ids; bad_token_ids = one-id sequences.
        phases: a dict that receives HIP events on the launch stream around the packed prefill, the step-graph
        capture and the decode steps ("t0", "prefill", "capture", "steps") plus the step count and the session's
        row lengths, for timing the leg's phases without a host sync inside it.
        """
        ev = (lambda: torch.cuda.Event(enable_timing=True)) if phases is not None else None
        if ev is not None:
            phases["t0"] = ev()
            phases["t0"].record()
        sess = DecodeSession(self, prompts, weights16, layers_to_heads, max_new_tokens,
                             [[int(t)] for t in bad_token_ids] + [list(map(int, s)) for s in bad_words_ids],
                             repetition_penalty)
        sess.prefill()
        if ev is not None:
            phases["prefill"] = ev()
            phases["prefill"].record()
        steps = max_new_tokens - 1
        if use_graph and steps > 0:
            sess.capture()
        if ev is not None:
            phases["capture"] = ev()
            phases["capture"].record()
        eos = torch.tensor(list(eos_ids) or [-1], device=self.device)
        n_steps = 0
        for t in range(steps):
            sess.step(use_graph)
            n_steps += 1
            # every 8 steps: stop once every row has produced an EOS (one host sync per check)
            if stop_on_eos and eos_ids and (t % 8 == 7 or t == steps - 1):
                if bool(torch.isin(sess.generated(), eos).any(1).all()):
                    break
        if ev is not None:
            phases["steps"] = ev()
            phases["steps"].record()
            phases["n_steps"] = n_steps
            phases["lens"] = list(sess.lens)
            phases["prefix"] = int(getattr(sess, "prefix", 0))
            phases["shared_read"] = int(sess.shared_read) // 32 * 32      # rows the step's attention reads once
        out = []
        gen = sess.generated().cpu().tolist()
        for row in gen:
            row = row[:max_new_tokens]
            if eos_ids:
                for i, tok in enumerate(row):
                    if tok in eos_ids:
                        row = row[:i + 1]
                        break
            out.append(row)
        return out


# Decode-step projections on the split-K matrix-core GEMM (cram_gemm_splitk): rows = the batch (one token per
# sequence), so a 256-row output tile spans every row and K is cut into ranges until the grid fills the chip.
# Measured against hipBLASLt with the decode pins (tools/decode_gemm_probe.py, B = 256, weights streamed cold,
# profiles/r03/decode_gemm_probe_*.jsonl): only the long-K down projection wins (Llama-3 N 4096 x K 14336: 55.9 vs
# 62.9 us at 8 ranges = 128 workgroups); at K <= N (q/k/v, o_proj, gate/up, lm_head) the fp32 partial slabs and
# their combine cost more than the library loses, so those stay on F.linear.  CRAM_DECODE_GEMM=0 turns it off (A/B).
DECODE_GEMM_MAX_ROWS = int(os.environ.get("CRAM_DECODE_GEMM_MAX_ROWS", "1024"))  # A/B override
DECODE_GEMM_TARGET_WGS = 128
DECODE_GEMM_MIN_K_OVER_N = 2
DECODE_QKV_SPLIT_MAX_ROWS = 192
DECODE_MLP_W4_MIN_ROWS = int(os.environ.get("CRAM_DECODE_MLP_W4_MIN_ROWS", "384"))
DECODE_SPLIT_ROW_TILES = os.environ.get("CRAM_DECODE_SPLIT_ROW_TILES", "1") == "1"   # A/B (decode_splits)


def decode_splits(N: int, K: int, rows: int) -> int:
    """K ranges for one decode projection ([rows, K] x [N, K]^T), or 0 for F.linear: for long-K shapes
    (K >= DECODE_GEMM_MIN_K_OVER_N * N) the count that brings N / 256 column tiles x ranges nearest
    DECODE_GEMM_TARGET_WGS with ranges of >= 256 columns of K (the same count at every row count up to
    DECODE_GEMM_MAX_ROWS)."""
    if os.environ.get("CRAM_DECODE_GEMM", "1") == "0" or rows > DECODE_GEMM_MAX_ROWS or N % 256 or K % 64:
        return 0
    if K < DECODE_GEMM_MIN_K_OVER_N * N and os.environ.get("CRAM_DECODE_GEMM") != "all":
        return 0
    tiles = N // 256          # column tiles; the row tiles (rows > 256) are not counted: 8 ranges won at both 256 and
    best = 0                  # 512 rows (profiles/r03/s5_m512/probe_*.jsonl: Llama-3 down 67 vs 93 us at 4 ranges)
    # at <= 192 rows more ranges pay: Llama-3 down at 129 rows 41.9 us at 14 ranges (224 workgroups) vs 48.0 at 8
    # (profiles/r04/dec129/)
    target = DECODE_GEMM_TARGET_WGS if rows > DECODE_QKV_SPLIT_MAX_ROWS else 224
    if rows > 512 and DECODE_SPLIT_ROW_TILES:
        # beyond 512 rows the row tiles multiply the grid (and the fp32 partial slabs the combine reads): count them
        # and aim at one workgroup per CU -- down_proj at 1,000 rows over 4 K ranges on the 4-wave kernel (256
        # workgroups) instead of hipBLASLt's 128 x 128 tiles: config 2 steps 35.0 -> 34.3 ms, config 4 (Qwen2-7B)
        # 27.3 -> 25.7 ms, same box (profiles/r06/s2/decode_down_split_ab.txt); the column-tile rule alone gave 8
        # ranges (512 workgroups, twice the partial bytes) and lost there (34.9 ms)
        tiles *= -(-rows // 256)
        target = 256
    for s in range(1, K // 256 + 1):
        if K % (64 * s):
            continue
        if not best or abs(tiles * s - target) < abs(tiles * best - target):
            best = s
    return best


# Decode-step projections on cram_gemm_small (128 x 128 tiles, K split so the grid fills the CUs) at one 128-row
# activation tile: config 5's batch and every GPU's share of NQ-1000 at 8 GPUs.  Measured at 128 rows, Llama-3 widths
# (tools/decode_gemm_probe.py --M 128, profiles/r05/dec128/): q/k/v 22.8 vs 26.3 us (hipBLASLt), o_proj 18.8 vs 24.6,
# down_proj 34.6 vs 47.2 (the 8-wave split-K); gate/up (61-63 vs 60) and lm_head (the 4-wave kernel, 206 vs 246) stay.
# At 512 rows it loses (q/k/v 43-52 vs 42): a 128 x 128 tile moves twice the bytes per MFMA of a 256 x 256 one, and a
# CU pulls only ~30 GB/s from beyond its L2.
DECODE_SMALL_MAX_ROWS = 128


def small_splits(N: int, K: int, rows: int) -> int:
    """K ranges of cram_gemm_small for one decode projection, or 0 (not routed there): the most ranges that keep
    N / 128 column tiles x ranges within the 256 CUs with >= 4 K-tiles per range."""
    if (os.environ.get("CRAM_DECODE_GEMM", "1") == "0" or rows > DECODE_SMALL_MAX_ROWS or N % 128 or K % 64):
        return 0
    ntn, kt = N // 128, K // 64
    best = 0
    for s in range(1, kt + 1):
        if kt % s == 0 and ntn * s <= 256 and kt // s >= 4:
            best = s
    return best


def decode_attn_splits(B: int, num_kv_heads: int, S_max: int) -> int:
    """Split-S count of the decode attention: enough (batch row, kv head) work items x splits to cover ~512
    workgroups, at most 16 splits and at least 256 keys per split; long rows (>= 4096 keys) take at least 2 while
    there are fewer than 2048 work items (config 5, B = 129 x 8 kv heads, 8.4k keys: 5.54 -> 5.77 TB/s;
    B = 512 x 1k keys stays at 1 split: 2 measured 0.91x; tools/prof_decode.py, profiles/r04/dsplit/)."""
    splits = max(1, min(16, math.ceil(512 / max(1, B * num_kv_heads))))
    if S_max >= 4096 and B * num_kv_heads < 2048:
        splits = max(splits, 2)
    return max(1, min(splits, S_max // 256))


class DecodeSession:
    """Static-shape state of one batched greedy decode (KV cache, bias, token buffers)."""

    def __init__(self, eng: CrAMEngine, prompts, weights16, layers_to_heads, max_new_tokens, bad_words=(),
                 repetition_penalty: float = 1.0):
        sp = eng.spec
        self.eng = eng
        self.B = len(prompts)
        self.lens = [int(p.numel()) for p in prompts]
        self.S_max = max(self.lens) + max_new_tokens
        self.S_max = (self.S_max + 63) // 64 * 64
        dev = eng.device
        self.prompts = [p.reshape(-1).to(dev) for p in prompts]
        self.cb = CredibilityBias.build(list(weights16), layers_to_heads, sp.num_layers, sp.num_heads, dev,
                                        eng.dtype, s_cap=self.S_max)
        self.k_cache = torch.zeros((sp.num_layers, self.B, sp.num_kv_heads, self.S_max, sp.head_dim),
                                   dtype=eng.dtype, device=dev)
        self.v_cache = torch.zeros_like(self.k_cache)
        self.max_new = max_new_tokens
        self.tokens = torch.zeros(self.B, dtype=torch.long, device=dev)
        self.pos = torch.tensor(self.lens, dtype=torch.long, device=dev)          # position of the token being fed
        self.seq_lens = torch.tensor(self.lens, dtype=torch.int32, device=dev)     # keys visible after the write
        self.out = torch.zeros((self.B, max_new_tokens), dtype=torch.long, device=dev)
        self.t = torch.zeros((), dtype=torch.long, device=dev)                    # next output column
        # bad words (transformers' NoBadWordsLogitsProcessor): one-id sequences are banned at every step; a sequence of
        # n > 1 ids bans its last id while the row's last n - 1 ids (prompt + generated, kept in `hist`) equal its first
        # n - 1 -- all on the device, inside the captured step
        single = sorted({s[0] for s in bad_words if len(s) == 1})
        multi = sorted({tuple(s) for s in bad_words if len(s) > 1})
        if any(len(s) == 0 for s in bad_words):
            raise ValueError("empty bad-words sequence")
        self.bad = torch.tensor(single, dtype=torch.long, device=dev) if single else None
        self.bw_pre = self.bw_valid = self.bw_last = self.hist = None
        if multi:
            Lm = max(len(s) for s in multi) - 1
            pre = torch.full((len(multi), Lm), -1, dtype=torch.long)
            valid = torch.zeros((len(multi), Lm), dtype=torch.bool)
            for i, s in enumerate(multi):                 # right-aligned: column Lm - 1 is the id just before
                pre[i, Lm - (len(s) - 1):] = torch.tensor(s[:-1])
                valid[i, Lm - (len(s) - 1):] = True
            hist = torch.full((self.B, Lm), -1, dtype=torch.long)
            for b, p in enumerate(self.prompts):
                tail = p[-Lm:].cpu()
                hist[b, Lm - tail.numel():] = tail
            # a sequence longer than the row's ids so far never matches (HF skips it): the -1 fill matches no id
            self.bw_pre, self.bw_valid = pre.to(dev), valid.to(dev)
            self.bw_last = [s[-1] for s in multi]
            self.hist = hist.to(dev)
        # repetition penalty (transformers RepetitionPenaltyLogitsProcessor): the set of ids each row has seen so
        # far (prompt + generated) as a [B, V] mask, updated inside the (graph-captured) step
        self.penalty = float(repetition_penalty)
        self.seen = None
        if self.penalty != 1.0:
            if self.penalty <= 0:
                raise ValueError("repetition_penalty must be > 0")
            self.seen = torch.zeros((self.B, eng.lm_head.shape[0]), dtype=torch.bool, device=dev)
            for b, p in enumerate(self.prompts):
                self.seen[b, p] = True
        self.splits = decode_attn_splits(self.B, sp.num_kv_heads, self.S_max)
        self.ws = (torch.empty(ops.decode_workspace_bytes(self.B, sp.num_heads, sp.head_dim, self.splits),
                               dtype=torch.uint8, device=dev) if self.splits > 1 else None)
        self.graph = None
        self.prefix = self.shared_read = 0          # set by prefill(): the batch's shared opening
        self.rows = torch.arange(self.B, device=dev)
        self.cos, self.sin = eng.rope_tables(self.S_max)
        # split-K plan of the step's projections (0 = F.linear) and one workspace shared by all of them (the
        # step's GEMMs run in stream order)
        D, F, qkv = sp.hidden, sp.intermediate, sp.q_size + 2 * sp.kv_size
        self.splits_gemm = {"qkv": decode_splits(qkv, D, self.B), "o": decode_splits(D, sp.q_size, self.B),
                            "gu": decode_splits(2 * F, D, self.B), "down": decode_splits(D, F, self.B)}
        if not self.splits_gemm["qkv"] and self.B <= DECODE_QKV_SPLIT_MAX_ROWS and os.environ.get("CRAM_DECODE_GEMM",
                                                                                                   "1") != "0":
            # one partly filled row tile (config 5: 129 rows): q/k/v over 8 K ranges, 28 vs 41 us on hipBLASLt's pick
            # (Llama-3, tools/decode_gemm_probe.py --M 129, profiles/r04/dec129/); o_proj / gate/up stay on the library
            self.splits_gemm["qkv"] = 8 if D % (64 * 8) == 0 and qkv % 256 == 0 else 0
        # gate/up + SiLU-mul on the 4-wave kernel at >= 384 rows for the Llama-3 MLP shape (N 28,672, K 4,096): 111.6 vs
        # 116.6 us for hipBLASLt + cram_silu_mul at 512 rows; it loses at 129 rows (86 vs 64) and on Qwen2's shape
        # (N 37,888, K 3,584: 167.8 vs 153.1; config 4 steps 13.9 -> 14.5 ms), profiles/r04/dec129/, decq/; the
        # interleaved weight is built here, outside the step graph
        # CRAM_DECODE_MLP_W4=1 / 0 forces it on / off at any shape the kernel takes (A/B of other shapes)
        # "auto": when the kernel's 256 x 256 tiles fill at least 3/4 of the CU waves they take -- Llama-3 at 512 and
        # 1,000 rows (224 / 448 tiles: 0.875), Qwen2-7B at 1,000 rows (592 tiles: 0.77; steps 25.5 -> 23.1 ms against
        # hipBLASLt + silu_mul, profiles/r06/s2/decode_qwen2_gateup_w4_ab.txt) but not at 512 (296 tiles: 0.58, the
        # column tail below)
        w4_env = os.environ.get("CRAM_DECODE_MLP_W4", "auto")
        gu_tiles = -(-self.B // 256) * (2 * sp.intermediate // 256)
        gu_fill = gu_tiles / (-(-gu_tiles // eng.num_cus) * eng.num_cus) if eng.device.type == "cuda" else 0.0
        self.mlp_w4 = (not self.splits_gemm["gu"] and self.B >= DECODE_MLP_W4_MIN_ROWS and eng.device.type == "cuda"
                       and (gu_fill >= 0.75 if w4_env == "auto" else w4_env == "1")
                       and eng._fused_mlp_ok(torch.empty((self.B, sp.hidden), dtype=eng.dtype, device="meta"))
                       and os.environ.get("CRAM_DECODE_GEMM", "1") != "0")
        # gate/up where the 4-wave kernel's 256 x 256 tiles spill just past one wave of the CUs (Qwen2-7B at 512 rows:
        # N 37,888 = 148 column tiles x 2 row tiles = 296 tiles = 1.16 waves, so the kernel took two tile times and
        # lost to hipBLASLt, 167.8 vs 153 us): the columns of one whole wave on it (+ SiLU-mul), the rest through the
        # split-K GEMM with K cut until the tail fills the CUs (+ SiLU-mul in its combine, on [gate; up] rows of the
        # tail).  CRAM_DECODE_MLP_TAIL=0 keeps the library (A/B).
        self.mlp_tail = None
        if (not self.mlp_w4 and not self.splits_gemm["gu"] and self.B >= DECODE_MLP_W4_MIN_ROWS
                and eng.device.type == "cuda" and os.environ.get("CRAM_DECODE_MLP_TAIL", "1") != "0"
                and os.environ.get("CRAM_DECODE_GEMM", "1") != "0"
                and eng._fused_mlp_ok(torch.empty((self.B, sp.hidden), dtype=eng.dtype, device="meta"))):
            ntm, ntn, cus = -(-self.B // 256), 2 * F // 256, eng.num_cus
            if cus < ntm * ntn < cus * 3 // 2 and cus % ntm == 0:
                c0 = (cus // ntm) * 128                  # output columns of the whole wave (a tile = 128 outputs)
                tail_tiles = ntm * -(-2 * (F - c0) // 256)
                kt = D // 64
                s_best = 0
                for sv in range(1, kt + 1):
                    if kt % sv == 0 and tail_tiles * sv <= cus and kt // sv >= 4:
                        s_best = sv
                if s_best and F - c0 >= 64:
                    self.mlp_tail = (c0, s_best)
        if self.mlp_w4 or self.mlp_tail:
            for lw in eng.layers:
                eng._gate_up_interleaved(lw)
                if self.mlp_tail:
                    eng._gate_up_tail(lw, self.mlp_tail[0])
        # lm_head on the 4-wave kernel (vocab % 256 == 0): 225 vs 290 us at 129 rows, 418 vs 457 at 512 (Llama-3)
        self.lm_w4 = (eng.device.type == "cuda" and eng.dtype in (torch.bfloat16, torch.float16)
                      and eng.lm_head.shape[0] % 256 == 0
                      and D % 64 == 0 and D >= 128 and os.environ.get("CRAM_DECODE_GEMM", "1") != "0")
        # one activation tile: q/k/v, o_proj and down_proj on cram_gemm_small with the K split that fills the CUs (the
        # split-K / library picks above are then unused for them)
        kin = {"qkv": D, "o": sp.q_size, "down": F}
        shapes = {"qkv": qkv, "o": D, "gu": 2 * F, "down": D}
        self.small = {k: small_splits(shapes[k], kin[k], self.B) for k in kin} if eng.device.type == "cuda" else {}
        self.small = {k: v for k, v in self.small.items() if v}
        for k in self.small:
            self.splits_gemm[k] = 0
        tail = [] if not self.mlp_tail else [(2 * (F - self.mlp_tail[0]), self.mlp_tail[1])]
        need = max([ops.gemm_splitk_workspace_bytes(self.B, shapes[k], v) for k, v in
                    list(self.splits_gemm.items()) + list(self.small.items()) if v]
                   + [ops.gemm_splitk_workspace_bytes(self.B, n, v) for n, v in tail] or [0])
        self.gemm_ws = torch.empty(need, dtype=torch.uint8, device=dev) if need else None

    def _proj(self, x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], key: str) -> torch.Tensor:
        if key in self.small:
            return ops.gemm_small(x, w, self.small[key], ops.GEMM_STORE, bias=b, workspace=self.gemm_ws)
        s = self.splits_gemm[key]
        if s:
            return ops.gemm_splitk(x, w, s, ops.GEMM_STORE, bias=b, workspace=self.gemm_ws)
        return ops.linear(x, w, b)

    def _mlp(self, x: torch.Tensor, lw: LayerW) -> torch.Tensor:
        s = self.splits_gemm["gu"]
        if self.mlp_tail:
            c0, st = self.mlp_tail
            F = self.eng.spec.intermediate
            x2 = x.reshape(-1, x.shape[-1])
            act = torch.empty((x2.shape[0], F), dtype=x.dtype, device=x.device)
            ops.gemm(x2, self.eng._gate_up_interleaved(lw)[:2 * c0], ops.GEMM_SILU_MUL, out=act[:, :c0])
            ops.gemm_splitk(x2, self.eng._gate_up_tail(lw, c0), st, ops.GEMM_SILU_MUL_CAT, workspace=self.gemm_ws,
                            out=act[:, c0:])
            act = act.view(*x.shape[:-1], F)
        elif self.mlp_w4:
            act = ops.gemm(x, self.eng._gate_up_interleaved(lw), ops.GEMM_SILU_MUL)
        elif s:
            act = ops.gemm_splitk(x, lw.wgu, s, ops.GEMM_SILU_MUL_CAT, workspace=self.gemm_ws)
        else:
            act = ops.silu_mul(ops.linear(x, lw.wgu), self.eng.spec.intermediate)
        return self._proj(act, lw.wd, None, "down")

    def _pick(self, logits: torch.Tensor, rows: Optional[slice] = None) -> torch.Tensor:
        """Greedy choice as transformers' generate makes it: fp32 logits, the repetition penalty (score / p where
        positive, score * p where negative, on the row's seen ids), bad words to -inf, argmax."""
        if self.seen is not None:
            x = logits.float()
            seen = self.seen if rows is None else self.seen[rows]
            logits = torch.where(seen, torch.where(x < 0, x * self.penalty, x / self.penalty), x)
        if self.bad is not None:
            logits = logits.index_fill(-1, self.bad, float("-inf"))
        if self.hist is not None:
            h = self.hist if rows is None else self.hist[rows]
            match = ((h[:, None, :] == self.bw_pre[None]) | ~self.bw_valid[None]).all(-1)        # [rows, sequences]
            logits = logits.clone() if self.bad is None else logits
            for i, t in enumerate(self.bw_last):
                logits[:, t] = torch.where(match[:, i], float("-inf"), logits[:, t])
        nxt = torch.argmax(logits, dim=-1)
        if self.hist is not None:                 # the rows' ids so far, shifted by the new one
            new = torch.cat([h[:, 1:], nxt[:, None]], 1)
            if rows is None:
                self.hist.copy_(new)
            else:
                self.hist[rows] = new
        if self.seen is not None:             # scatter of a scalar: no host tensor, capturable in the step graph
            (self.seen if rows is None else self.seen[rows]).scatter_(1, nxt[:, None], True)
        return nxt

    def shared_prefix(self) -> int:
        """Rows every prompt of the batch shares at its start, unbiased in every row (the credibility weights are 1
        there, so those rows' attention is the same in every prompt), each prompt keeping >= 1 row of its own; 0 when
        fewer than PREFIX_SHARE_MIN_ROWS."""
        if not PREFIX_SHARE or self.B < 2:
            return 0
        n = min(self.lens) - 1
        if n < PREFIX_SHARE_MIN_ROWS:
            return 0
        ids = torch.stack([p[:n] for p in self.prompts])
        diff = (ids != ids[:1]).any(0)
        p = int(diff.nonzero()[0, 0]) if bool(diff.any()) else n
        Wp = min(p, self.cb.W)
        if Wp > 0:
            nz = (self.cb.bias[:, :Wp] != 0).any(0)
            if bool(nz.any()):
                p = int(nz.nonzero()[0, 0])
        return p if p >= PREFIX_SHARE_MIN_ROWS else 0

    def _prefill_prefix(self, p: int):
        """The shared prefix once (rows 0..p-1 of prompt 0: causal, unbiased), its K/V of every layer into cache row
        0, then copied to every other row.  The projections run on the packed prefill's kernels whatever the prefix's
        row count (q/k/v + RoPE into the cache, o_proj / down_proj + residual, gate/up + SiLU-mul on the 4-wave GEMM,
        which rounds a row the same whatever M): the prefix rows' K/V then differ from a whole-prompt prefill's only
        where the attention kernel's 32-row blocks fall differently."""
        eng, sp = self.eng, self.eng.spec
        h = eng.embed[self.prompts[0][:p]]
        m = None
        prev = eng.fused_any_rows, eng.no_tail_split
        eng.fused_any_rows, eng.no_tail_split = True, True
        try:
            for l, lw in enumerate(eng.layers):
                if m is None:
                    x = ops.rmsnorm(h, lw.ln1, sp.eps)
                else:
                    h, x = ops.rmsnorm(m, lw.ln1, sp.eps, residual=h)
                kc, vc = self.k_cache[l][:1].transpose(1, 2), self.v_cache[l][:1].transpose(1, 2)
                if eng._fused_qkv_ok(x, lw):
                    y = ops.gemm_rope(x, lw.wqkv, sp.num_heads, sp.num_kv_heads, sp.head_dim, self.cos, self.sin, p,
                                      rows=p, kout=kc, vout=vc, row0=0, keep_k=True, bias=lw.bqkv)
                else:
                    y = ops.linear(x, lw.wqkv, lw.bqkv)
                    ops.rope_split(y, sp.num_heads, sp.num_kv_heads, sp.head_dim, self.cos, self.sin, p, kc, vc, 0,
                                   keep_k=True)
                self.k_cache[l][1:, :, :p] = self.k_cache[l][:1, :, :p]
                self.v_cache[l][1:, :, :p] = self.v_cache[l][:1, :, :p]
                if l == sp.num_layers - 1:              # the last layer's K/V are all the prefix contributes
                    break
                q = y[:, :sp.q_size].unflatten(-1, (sp.num_heads, sp.head_dim))[None]
                k = y[:, sp.q_size:sp.q_size + sp.kv_size].unflatten(-1, (sp.num_kv_heads, sp.head_dim))[None]
                v = y[:, sp.q_size + sp.kv_size:].unflatten(-1, (sp.num_kv_heads, sp.head_dim))[None]
                a = eng.attention(q, k, v)
                h, x2 = eng.o_proj_norm(a.reshape(p, sp.q_size), lw, h)
                h, m = eng.mlp_residual(x2, lw, h)
        finally:
            eng.fused_any_rows, eng.no_tail_split = prev

    def prefill(self, max_rows: int = PREFILL_CHUNK_ROWS):
        """All prompts in packed varlen passes of at most ``max_rows`` tokens each (GEMM M = the chunk's token
        count rounded to 256 rows; attention per sequence through cram_attn_prefill_varlen; K/V scattered into
        the cache).  Chunks of the sweep's GEMM size run the GEMMs at the same rate as one huge pass, keep the
        activations ~8x smaller and — every chunk having the same shape bound — let the caching allocator reuse
        the same blocks across chunks and calls (one 231k-row pass made it map fresh multi-GB segments, a ~1 s
        host stall per call)."""
        b0 = 0
        self.prefix = p = self.shared_prefix()
        self.shared_read = p if SHARED_DECODE_READ else 0
        with gemm_tune.pinned():
            if p:
                self._prefill_prefix(p)
            while b0 < self.B:
                b1, rows = b0, 0
                while b1 < self.B and (b1 == b0 or rows + self.lens[b1] - p <= max_rows):
                    rows += self.lens[b1] - p
                    b1 += 1
                self._prefill_chunk(b0, b1, p)
                b0 = b1
        self.out[:, 0] = self.tokens
        self.t.fill_(1)

    def _prefill_chunk(self, b0: int, b1: int, p: int = 0):
        """Prompts b0..b1-1 from row p on (p = the shared prefix already in the cache, or 0), packed."""
        eng, sp = self.eng, self.eng.spec
        dev = eng.device
        lens = [n - p for n in self.lens[b0:b1]]
        total = sum(lens)
        Mp = padded_rows(total, sp)
        offs = [0]
        for n in lens:
            offs.append(offs[-1] + n)
        cu = torch.tensor(offs, dtype=torch.int32).to(dev, non_blocking=True)
        pos = torch.cat([torch.arange(p, p + n, dtype=torch.long) for n in lens]).to(dev, non_blocking=True)
        bidx = torch.cat([torch.full((n,), b, dtype=torch.long) for b, n in enumerate(lens, b0)]).to(
            dev, non_blocking=True)
        h = torch.empty((Mp, sp.hidden), dtype=eng.dtype, device=dev)
        h[:total] = eng.embed[torch.cat([t[p:] for t in self.prompts[b0:b1]])]
        if Mp > total:
            h[total:].zero_()
        bias = self.cb.bias[b0:b1]
        last = cu[1:].long() - 1                     # each sequence's last row: the only one the logits need
        # the attention output of every layer: the kernels write rows :total, so the pad rows o_proj reads are zeroed
        # once per chunk, not once per layer
        a = torch.empty((Mp, sp.q_size), dtype=eng.dtype, device=dev)
        if Mp > total:
            a[total:].zero_()
        m = None                                     # pending MLP output: layer output = h + m (add fused below)
        for l, lw in enumerate(eng.layers):
            if m is None:
                x = ops.rmsnorm(h, lw.ln1, sp.eps)
            else:
                h, x = ops.rmsnorm(m, lw.ln1, sp.eps, residual=h)
            # q roped in place, roped k and v written straight into the cache rows (sequence bidx, position pos) of
            # this layer; k also kept in place when the packed attention reads it there (no shared prefix)
            kc, vc = self.k_cache[l].transpose(1, 2), self.v_cache[l].transpose(1, 2)
            if eng._fused_qkv_ok(x, lw):
                y = ops.gemm_rope(x, lw.wqkv, sp.num_heads, sp.num_kv_heads, sp.head_dim, self.cos, self.sin, 1,
                                  rows=total, kout=kc, vout=vc, row0=0, pos=pos, dst_b=bidx, keep_k=p == 0,
                                  bias=lw.bqkv)
            else:
                y = ops.linear(x, lw.wqkv, lw.bqkv)
                ops.rope_split(y[:total], sp.num_heads, sp.num_kv_heads, sp.head_dim, self.cos, self.sin, 1, kc, vc,
                               0, pos=pos, dst_b=bidx, keep_k=p == 0)
            yr = y[:total]
            q = yr[:, :sp.q_size].view(total, sp.num_heads, sp.head_dim)
            if l == sp.num_layers - 1:
                # last layer: every row's K/V is in the cache now and only the last rows feed the logits, so their
                # attention is one decode-kernel call over the cache and o_proj / MLP run on those rows alone (the
                # other rows' last-layer outputs are never read: 2.7 % of the prefill's FLOPs)
                a = ops.attn_decode(q[last], self.k_cache[l][b0:b1], self.v_cache[l][b0:b1], scale=eng.scale,
                                    seq_lens=self.seq_lens[b0:b1], bias=bias, enable=self.cb.enable[l, b0:b1],
                                    W=self.cb.W, num_splits=self.splits, workspace=self.ws,
                                    shared_rows=self.shared_read)
                h, x2 = ops.rmsnorm(ops.linear(a.flatten(-2), lw.wo), lw.ln2, sp.eps, residual=h[last])
                m = eng.mlp(x2, lw)
                break
            k = yr[:, sp.q_size:sp.q_size + sp.kv_size].view(total, sp.num_kv_heads, sp.head_dim)
            v = yr[:, sp.q_size + sp.kv_size:].view(total, sp.num_kv_heads, sp.head_dim)
            if p:                                    # keys: the cached prefix, then the suffix's own rows
                ops.attn_prefill_varlen_cached(q, kc[b0:b1], vc[b0:b1], cu, max(lens), p, scale=eng.scale, bias=bias,
                                               enable=self.cb.enable[l, b0:b1], W=self.cb.W,
                                               out=a[:total].view(total, sp.num_heads, sp.head_dim))
            else:
                ops.attn_prefill_varlen(q, k, v, cu, max(lens), scale=eng.scale, bias=bias,
                                        enable=self.cb.enable[l, b0:b1], W=self.cb.W,
                                        out=a[:total].view(total, sp.num_heads, sp.head_dim))
            h, x2 = eng.o_proj_norm(a, lw, h)
            h, m = eng.mlp_residual(x2, lw, h)
        hn = ops.rmsnorm(h, eng.norm, sp.eps) if m is None else ops.rmsnorm(m, eng.norm, sp.eps, residual=h)[1]
        self.tokens[b0:b1] = self._pick(ops.linear(hn, eng.lm_head), slice(b0, b1))

    def _step_body(self):
        eng, sp = self.eng, self.eng.spec
        h = eng.embed[self.tokens][:, None]                      # [B, 1, D]
        self.seq_lens.add_(1)
        m = None                    # pending MLP output: the residual add runs inside the next RMSNorm
        for l, lw in enumerate(eng.layers):
            if m is None:
                x = eng.rmsnorm(h, lw.ln1)
            else:
                h, x = eng.add_rmsnorm(m, h, lw.ln1)
            y = self._proj(x, lw.wqkv, lw.bqkv, "qkv")         # [B, 1, (Hq + 2 Hkv) d]
            # q roped in place; the new token's roped k and its v straight into cache row pos of every sequence
            ops.rope_split(y, sp.num_heads, sp.num_kv_heads, sp.head_dim, self.cos, self.sin, 1,
                           self.k_cache[l].transpose(1, 2), self.v_cache[l].transpose(1, 2), 0, pos=self.pos,
                           dst_b=self.rows)
            q = y[..., :sp.q_size].unflatten(-1, (sp.num_heads, sp.head_dim))
            # the batch's shared opening (prefilled once, copied into every row) read from row 0 (bit-identical)
            a = ops.attn_decode(q[:, 0], self.k_cache[l], self.v_cache[l], scale=eng.scale, seq_lens=self.seq_lens,
                                bias=self.cb.bias, enable=self.cb.enable[l], W=self.cb.W, num_splits=self.splits,
                                workspace=self.ws, shared_rows=self.shared_read)
            h, x2 = eng.add_rmsnorm(self._proj(a.flatten(-2)[:, None], lw.wo, None, "o"), h, lw.ln2)
            m = self._mlp(x2, lw)
        _, hn = eng.add_rmsnorm(m[:, 0], h[:, 0], eng.norm)
        nxt = self._pick(ops.gemm(hn, eng.lm_head) if self.lm_w4 else ops.linear(hn, eng.lm_head))
        self.tokens.copy_(nxt)
        self.out.index_copy_(1, self.t.view(1), nxt[:, None])
        self.t.add_(1)
        self.pos.add_(1)

    def capture(self):
        s = torch.cuda.Stream(self.eng.device)
        s.wait_stream(torch.cuda.current_stream(self.eng.device))
        # warm the allocator / kernels on a side stream, then restore the state it advanced
        snap = (self.tokens.clone(), self.pos.clone(), self.seq_lens.clone(), self.t.clone(), self.out.clone(),
                None if self.seen is None else self.seen.clone(), None if self.hist is None else self.hist.clone())
        with gemm_tune.pinned(decode=True), torch.cuda.stream(s):
            self._step_body()
        torch.cuda.current_stream(self.eng.device).wait_stream(s)
        self.tokens.copy_(snap[0]); self.pos.copy_(snap[1]); self.seq_lens.copy_(snap[2])
        self.t.copy_(snap[3]); self.out.copy_(snap[4])
        if self.seen is not None:
            self.seen.copy_(snap[5])
        if self.hist is not None:
            self.hist.copy_(snap[6])
        self.graph = torch.cuda.CUDAGraph()
        with gemm_tune.pinned(decode=True), torch.cuda.graph(self.graph):
            self._step_body()

    def step(self, use_graph=True):
        if use_graph and self.graph is not None:
            self.graph.replay()
        else:
            with gemm_tune.pinned(decode=True):
                self._step_body()

    def generated(self) -> torch.Tensor:
        return self.out
