"""transformers AttentionInterface registration: "cram_hip".

This replaces the reference's plug-point, a forward-pre-hook on
model.layers.{l}.self_attn that rewrites attention_mask
(re_weighting.py:118-124, :163-168), plus the SDPA call the mask flows into
(transformers 5.15 sdpa_attention_forward).  With config._attn_implementation
set to "cram_hip" transformers builds no mask at all (the name is not in the
mask registry) and calls `cram_attention_forward` with the strided q/k/v of each
layer; the credibility descriptor is attached to the attention modules by
`reweighting(...)` for the duration of a call.
"""
from __future__ import annotations

import contextlib
import math
from typing import Optional

import torch

from . import ops
from .bias import CredibilityBias

IMPL_NAME = "cram_hip"
_registered = False


def _num_splits(B: int, Hkv: int, S: int) -> int:
    s = max(1, min(16, math.ceil(512 / max(1, B * Hkv))))
    return max(1, min(s, S // 256))


def cram_attention_forward(module: torch.nn.Module, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor,
                           attention_mask: Optional[torch.Tensor], scaling: Optional[float] = None,
                           dropout: float = 0.0, **kwargs):
    """q [B, Hq, Tq, d], k/v [B, Hkv, S, d] -> ([B, Tq, Hq, d], None) on the HIP kernels."""
    if attention_mask is not None:
        raise NotImplementedError("cram_hip attention builds its own causal mask; padded batches are not supported "
                                  "on the transformers path (use CrAMEngine for batched prompts)")
    if dropout != 0.0:
        raise NotImplementedError("cram_hip attention is inference-only")
    if scaling is None:
        scaling = query.shape[-1] ** -0.5
    cb: Optional[CredibilityBias] = getattr(module, "_cram_bias", None)
    bias = enable = None
    W = 0
    if cb is not None:
        bias, enable, W = cb.bias, cb.enable[module.layer_idx], cb.W
    # bf16 / fp16 models run in their own dtype; fp32 ones (GPT-2 checkpoints) on bf16 operands
    dt = query.dtype if query.dtype in ops.DTYPES else torch.bfloat16
    q, k, v = (t if t.dtype == dt else t.to(dt) for t in (query, key, value))
    B, Hq, Tq, d = q.shape
    if Tq == 1:
        S = k.shape[2]
        out = ops.attn_decode(q[:, :, 0], k, v, scale=scaling, bias=bias, enable=enable, W=W,
                              num_splits=_num_splits(B, k.shape[1], S))
        out = out.view(B, 1, Hq, d)
    else:
        out = ops.attn_prefill(q, k, v, scale=scaling, bias=bias, enable=enable, W=W)
    if out.dtype != query.dtype:
        out = out.to(query.dtype)
    return out, None


def register() -> str:
    """Register "cram_hip" with transformers (idempotent)."""
    global _registered
    if not _registered:
        from transformers import AttentionInterface
        AttentionInterface.register(IMPL_NAME, cram_attention_forward)
        _registered = True
    return IMPL_NAME


def attention_modules(model):
    """(layer index, attention module) of a decoder-only transformers model: `model.layers.{l}.self_attn`
    (Llama / Qwen2 / Mistral families, re_weighting.py:120) or `transformer.h.{l}.attn` (GPT-2, which the
    reference's hook path cannot address)."""
    base = model.base_model
    if hasattr(base, "layers"):
        for l, layer in enumerate(base.layers):
            yield l, layer.self_attn
    elif hasattr(base, "h"):
        for l, blk in enumerate(base.h):
            yield l, blk.attn
    else:
        raise NotImplementedError(f"no known attention-module layout for {type(model).__name__}")


@contextlib.contextmanager
def reweighting(model, cb: Optional[CredibilityBias]):
    """Attach a CredibilityBias to every attention module of `model` for the duration of the block.

    Equivalent to registering the reference's forward-pre-hooks on every layer
    listed in the enable mask and removing them afterwards — but removal is
    guaranteed (the reference has no try/finally, re_weighting.py:132-137).
    """
    mods = [m for _, m in attention_modules(model)]
    for m in mods:
        m._cram_bias = cb
    try:
        yield
    finally:
        for m in mods:
            m._cram_bias = None
