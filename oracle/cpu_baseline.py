"""ORACLE — test infrastructure only.  The timed CPU baseline of bench.py.

The reference's IE sweep on the host cores (re_weighting.py:152-175): a
transformers Llama model on the CPU, the restated dense-mask forward-pre-hook
(oracle.hook_ref), one full forward with full-vocab logits per (layer, head)
unit and a .item() per unit.  Weights are copied from the GPU engine so both
sides run the same network.  Only bench.py's cpu_baseline leg calls this.
"""
from __future__ import annotations

import os
import time

import torch

from . import hook_ref


def hf_model_from_engine(eng, rope_theta: float = 500000.0):
    """A transformers LlamaForCausalLM on the CPU holding the engine's weights (in the engine's dtype)."""
    from transformers import LlamaConfig, LlamaForCausalLM
    sp = eng.spec
    cfg = LlamaConfig(vocab_size=sp.vocab, hidden_size=sp.hidden, intermediate_size=sp.intermediate,
                      num_hidden_layers=sp.num_layers, num_attention_heads=sp.num_heads,
                      num_key_value_heads=sp.num_kv_heads, head_dim=sp.head_dim, rms_norm_eps=sp.eps,
                      rope_theta=rope_theta, max_position_embeddings=8192, tie_word_embeddings=False)
    cfg._attn_implementation = "sdpa"
    prev = torch.get_default_dtype()
    torch.set_default_dtype(eng.dtype)
    try:
        with torch.device("meta"):
            model = LlamaForCausalLM(cfg)
    finally:
        torch.set_default_dtype(prev)
    model = model.to_empty(device="cpu")
    q, kv = sp.q_size, sp.kv_size
    with torch.no_grad():
        model.model.embed_tokens.weight.copy_(eng.embed.cpu())
        model.model.norm.weight.copy_(eng.norm.cpu())
        model.lm_head.weight.copy_(eng.lm_head.cpu())
        for blk, lw in zip(model.model.layers, eng.layers):
            wqkv = lw.wqkv.cpu()
            blk.self_attn.q_proj.weight.copy_(wqkv[:q])
            blk.self_attn.k_proj.weight.copy_(wqkv[q:q + kv])
            blk.self_attn.v_proj.weight.copy_(wqkv[q + kv:])
            blk.self_attn.o_proj.weight.copy_(lw.wo.cpu())
            wgu = lw.wgu.cpu()
            blk.mlp.gate_proj.weight.copy_(wgu[:sp.intermediate])
            blk.mlp.up_proj.weight.copy_(wgu[sp.intermediate:])
            blk.mlp.down_proj.weight.copy_(lw.wd.cpu())
            blk.input_layernorm.weight.copy_(lw.ln1.cpu())
            blk.post_attention_layernorm.weight.copy_(lw.ln2.cpu())
        rot = model.model.rotary_emb
        rot.inv_freq = eng.inv_freq.detach().float().cpu().clone()
        if hasattr(rot, "original_inv_freq"):
            rot.original_inv_freq = rot.inv_freq.clone()
    model.eval()
    return model


def cores() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


@torch.no_grad()
def time_ie_units(model, ids: torch.Tensor, w16: torch.Tensor, answer_ids: torch.Tensor, units) -> dict:
    """Reference-algorithm IE units on the CPU: one hooked full forward + .item() per (layer, head)."""
    torch.set_num_threads(cores())
    lw = hook_ref.log_weight(w16.reshape(1, -1).cpu())
    ids = ids.reshape(1, -1).cpu()
    am = torch.ones_like(ids)
    ori = hook_ref.answer_logit_sum(model(input_ids=ids, attention_mask=am).logits, answer_ids)
    t0 = time.perf_counter()
    vals, per = [], []
    for (l, h) in units:
        t1 = time.perf_counter()
        hs = hook_ref.register_hooks(model, {l: [h]}, lw)
        try:
            cur = hook_ref.answer_logit_sum(model(input_ids=ids, attention_mask=am).logits, answer_ids)
        finally:
            for x in hs:
                x.remove()
        vals.append((ori - cur).item())
        per.append(time.perf_counter() - t1)
    dt = time.perf_counter() - t0
    srt = sorted(per)
    return {"units": len(units), "seconds": dt, "units_per_s": len(units) / dt, "cores": cores(),
            "ie": vals, "unit_seconds": per,
            "spread": {"min_s": srt[0], "median_s": srt[len(srt) // 2], "max_s": srt[-1]}}


def sample_units(num_layers: int, num_heads: int, n: int):
    """n (layer, head) units spread over the layers (first, last, middle, quarters, ...) and heads."""
    fr = [0.0, 1.0, 0.5, 0.25, 0.75, 0.125, 0.625, 0.375, 0.875]
    out = []
    for i in range(n):
        l = round(fr[i % len(fr)] * (num_layers - 1)) if i < len(fr) else (i * 7) % num_layers
        out.append((int(l), int((i * 11 + 3) % num_heads)))
    return out
