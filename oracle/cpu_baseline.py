"""ORACLE — test infrastructure only.  The timed CPU baseline of bench.py.

Both halves of the metric on the host cores, through the reference's own
algorithm: a transformers Llama / Qwen2 model on the CPU with the restated
dense-mask forward-pre-hook (oracle.hook_ref):
  * IE sweep (re_weighting.py:152-175): one full forward with full-vocab logits
    per (layer, head) unit and a .item() per unit;
  * reweighted decode (re_weighting.py:115-138): hooks on the selected heads,
    then greedy `generate` at batch 1.
Weights are copied from the GPU engine so both sides run the same network.
Only bench.py's cpu_baseline legs call this.
"""
from __future__ import annotations

import os
import time

import torch

from . import hook_ref


def hf_model_from_engine(eng, rope_theta: float = 500000.0):
    """A transformers LlamaForCausalLM (Qwen2ForCausalLM for the qwen2 family, q/k/v biases included) on the CPU
    holding the engine's weights (in the engine's dtype).  The rotary table is copied from the engine, so
    rope_theta only fills the config."""
    sp = eng.spec
    common = dict(vocab_size=sp.vocab, hidden_size=sp.hidden, intermediate_size=sp.intermediate,
                  num_hidden_layers=sp.num_layers, num_attention_heads=sp.num_heads,
                  num_key_value_heads=sp.num_kv_heads, head_dim=sp.head_dim, rms_norm_eps=sp.eps, rope_theta=rope_theta,
                  max_position_embeddings=16384, tie_word_embeddings=False)
    if sp.family == "qwen2":
        from transformers import Qwen2Config as Cfg, Qwen2ForCausalLM as Model
        cfg = Cfg(**common)
    else:
        from transformers import LlamaConfig as Cfg, LlamaForCausalLM as Model
        cfg = Cfg(**common)
    cfg._attn_implementation = "sdpa"
    prev = torch.get_default_dtype()
    torch.set_default_dtype(eng.dtype)
    try:
        with torch.device("meta"):
            model = Model(cfg)
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
            if lw.bqkv is not None:
                b = lw.bqkv.cpu()
                blk.self_attn.q_proj.bias.copy_(b[:q])
                blk.self_attn.k_proj.bias.copy_(b[q:q + kv])
                blk.self_attn.v_proj.bias.copy_(b[q + kv:])
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
def time_ie_units(model, ids: torch.Tensor, w16: torch.Tensor, answer_ids: torch.Tensor, units, log=None) -> dict:
    """Reference-algorithm IE units on the CPU: one hooked full forward + .item() per (layer, head).  log: called
    with a progress line every 8 units (the bench's stderr: a silent minute reads as a hang on the GPU box)."""
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
        if log is not None and len(per) % 8 == 0:
            log(f"cpu IE sample: {len(per)}/{len(units)} units at {time.perf_counter() - t0:.1f}s")
    dt = time.perf_counter() - t0
    srt = sorted(per)
    return {"units": len(units), "seconds": dt, "units_per_s": len(units) / dt, "cores": cores(),
            "ie": vals, "unit_seconds": per,
            "spread": {"min_s": srt[0], "median_s": srt[len(srt) // 2], "max_s": srt[-1]}}


def sample_units(num_layers: int, num_heads: int, n: int):
    """n (layer, head) units: whole layers of all heads (BASELINE.md's plan: 1 question x 2 layers x 32 heads = 64
    units), the layers taken in the spread order first, last, middle, quarters, ...; a count that is not a multiple
    of the head count ends with the first heads of one more layer.  (In the reference every unit is one full hooked
    forward whatever its layer, re_weighting.py:162-171, so the layers only spread the sample.)"""
    fr = [0.0, 1.0, 0.5, 0.25, 0.75, 0.125, 0.625, 0.375, 0.875]
    order = []
    for f in fr + [i / num_layers for i in range(num_layers)]:
        l = int(round(f * (num_layers - 1)))
        if l not in order:
            order.append(l)
    out = []
    for l in order:
        for h in range(num_heads):
            if len(out) == n:
                return out
            out.append((l, h))
    return out


@torch.no_grad()
def time_decode(model, ids: torch.Tensor, w16: torch.Tensor, layers_to_heads: dict, new_tokens: int = 100,
                sampled_steps: int = 8, layers: int = 0, log=None) -> dict:
    """The reference's reweighted decode of one question on the CPU (re_weighting.py:115-138): forward-pre-hooks
    on the selected heads (:118-124), greedy `generate` (:127-132).  Bounded sample: generate runs 1 + sampled_steps
    tokens (min_new_tokens keeps EOS from ending it early); a StoppingCriteria stamps the clock after every token,
    so the first stamp closes the prefill (+ the first token) and the rest are the per-token decode steps.  One
    question's time at `new_tokens` = prefill + (new_tokens - 1) x median step (linear extrapolation; the per-step
    attention cost grows by ~1 key per step, < 0.1 % of a ~900-token prompt's).

    layers = k > 0 (long prompts, where the hooked forward is minutes on the host: the dense [H, T, T] mask of every
    hooked layer): the sample runs the first k decoder layers only (their weights, their hooks) and the per-layer part
    of the time is scaled by L / k (embedding and the one-row lm_head ride along unscaled, a < 1 % under-count of the
    reference's time)."""
    from transformers import StoppingCriteria, StoppingCriteriaList
    torch.set_num_threads(cores())
    ids = ids.reshape(1, -1).cpu()
    lw = hook_ref.log_weight(w16.reshape(1, -1).cpu())
    stamps = []

    class _Stamp(StoppingCriteria):
        def __call__(self, input_ids, scores, **kwargs):
            stamps.append(time.perf_counter())
            if log is not None:
                log(f"cpu decode sample: token {len(stamps)} at {stamps[-1] - t0:.1f}s")
            return torch.zeros(input_ids.shape[0], dtype=torch.bool)

    n = 1 + max(1, int(sampled_steps))
    L = model.config.num_hidden_layers
    k = int(layers) if 0 < int(layers) < L else L
    full_layers = model.model.layers
    if k < L:
        model.model.layers = full_layers[:k]
        model.config.num_hidden_layers = k
        layers_to_heads = {l: v for l, v in layers_to_heads.items() if int(l) < k}
    hs = hook_ref.register_hooks(model, layers_to_heads, lw)
    try:
        t0 = time.perf_counter()
        out = model.generate(input_ids=ids, attention_mask=torch.ones_like(ids), do_sample=False, max_new_tokens=n,
                             min_new_tokens=n, stopping_criteria=StoppingCriteriaList([_Stamp()]), pad_token_id=0)
    finally:
        for h in hs:
            h.remove()
        model.model.layers = full_layers
        model.config.num_hidden_layers = L
    if len(stamps) != n or out.shape[1] != ids.shape[1] + n:
        raise RuntimeError(f"CPU decode sample produced {out.shape[1] - ids.shape[1]} tokens, {len(stamps)} stamps")
    scale = L / k
    prefill = (stamps[0] - t0) * scale
    steps = sorted((b - a) * scale for a, b in zip(stamps, stamps[1:]))
    med = steps[len(steps) // 2]
    per_q = prefill + (max(1, int(new_tokens)) - 1) * med
    return {"prefill_s": prefill, "step_s": {"min": steps[0], "median": med, "max": steps[-1]},
            "sampled_steps": len(steps), "seconds": stamps[-1] - t0, "question_s": per_q,
            "questions_per_s": 1.0 / per_q, "cores": cores(), "prompt_tokens": int(ids.shape[1]),
            "heads": sum(len(v) for v in layers_to_heads.values()), "layers_run": k, "layers": L}
