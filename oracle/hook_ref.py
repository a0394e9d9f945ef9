"""ORACLE — test infrastructure only.  CPU restatement of the reference hook path.

Each function restates one piece of /root/reference (cited file:line) in plain
torch/numpy on the CPU.  It is the checker for the HIP path and the timed CPU
baseline of bench.py; the product package (cram_amd) never imports it.
"""
from __future__ import annotations

from functools import partial
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

# utils/prompts_templates.py:5-6 ('qa' / 'with_contexts')
WITH_CONTEXTS = ("Given the following information: \n{paras}\nAnswer the following question based on the given "
                 "information or your internal knowledge with one or few words without the source.\n"
                 "Question: {question}\nAnswer: {answer}")
LLAMA3_SYSTEM = "You are a helpful assistant!"   # re_weighting.py:68-71
QWEN_SYSTEM = "You are a helpful assistant."     # re_weighting.py:83-86


def get_prompt(context: Sequence[str], question: str, answer: str = "") -> str:
    """utils/prompt.py:4-12 (type='with_contexts')."""
    body = "\n".join(f"Passage-{i}: {p}" for i, p in enumerate(context))
    return WITH_CONTEXTS.format(question=question, paras=body, answer=answer)


def chat_prompt(tokenizer, model_name: str, paras: Sequence[str], question: str, answer: str = "") -> Tuple[str, bool]:
    """re_weighting.py:64-95: the text that gets tokenised and whether special tokens are added."""
    if "Llama-3" in model_name or "Qwen" in model_name:
        system = LLAMA3_SYSTEM if "Llama-3" in model_name else QWEN_SYSTEM
        msgs = [{"role": "system", "content": system},
                {"role": "user", "content": get_prompt(paras, question, "")}]
        text = tokenizer.apply_chat_template(msgs, add_generation_prompt=True, tokenize=False)
        if answer != "":
            text += answer
        return text, "Llama-3" in model_name
    return get_prompt(paras, question, answer), True


def token_spans(prompt: str, paras: Sequence[str], offsets: Sequence[Tuple[int, int]]) -> List[Tuple[int, int]]:
    """re_weighting.py:100-110: inclusive token span of each 'Passage-i: <p>\\n' over offset starts."""
    spans = []
    starts = [int(o[0]) for o in offsets]
    for i, p in enumerate(paras):
        text = f"Passage-{i}: {p}\n"
        c0 = prompt.find(text)
        c1 = c0 + len(text) - 1
        t0 = t1 = None
        for t, s in enumerate(starts):
            if c0 >= s:
                t0 = t
            if c1 >= s:
                t1 = t
        if t0 is None or t1 is None:
            raise ValueError(f"passage {i} not found in prompt")
        spans.append((t0, t1))
    return spans


def weight_vector(T: int, spans: Sequence[Tuple[int, int]], scores: Sequence[float]) -> torch.Tensor:
    """re_weighting.py:99,111: fp16 [1, T] ones, then each span overwritten in passage order."""
    w = torch.ones((1, T), dtype=torch.float16)
    for (t0, t1), sc in zip(spans, scores):
        w[:, t0:t1 + 1] = torch.full((1, t1 + 1 - t0), float(sc)).to(torch.float16)
    return w


def log_weight(w16: torch.Tensor) -> torch.Tensor:
    """re_weighting.py:122,166: natural log evaluated on the fp16 tensor."""
    return torch.log(w16)


def edit_attention_mask(num_heads: int, hidden_states: torch.Tensor, attention_mask: Optional[torch.Tensor],
                        position_ids: torch.Tensor, lw: torch.Tensor, head_idx: Sequence[int]) -> torch.Tensor:
    """re_weighting.py:36-61: the dense [1, H, T, S] mask the forward-pre-hook writes."""
    W = lw.shape[-1]
    dt = hidden_states.dtype
    if attention_mask is None:
        T = hidden_states.shape[1]
        S = int(position_ids[0][-1]) + 1
        if T == 1:
            mask = torch.zeros((1, 1, 1, S), dtype=dt, device=hidden_states.device)
        else:
            mask = torch.triu(torch.full((T, S), torch.finfo(dt).min, dtype=dt, device=hidden_states.device),
                              diagonal=1)[None, None]
    else:
        mask = attention_mask.clone()
    if mask.shape[1] == 1:
        mask = mask.repeat(1, num_heads, 1, 1)
    mask = mask.clone()
    B, H, T, S = mask.shape
    row = lw.reshape(-1).to(device=mask.device, dtype=dt)
    rows = row.expand(T, W)
    for h in head_idx:
        sub = mask[:, h, :, :W]
        allowed = sub == 0
        sub[allowed] = rows.unsqueeze(0).expand(B, T, W)[allowed]
    return mask


def sdpa_ref(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, mask: Optional[torch.Tensor],
             scale: float) -> torch.Tensor:
    """softmax(q k^T * scale + mask) v in float64 (GQA by repeating kv heads).

    q [B, Hq, T, d], k/v [B, Hkv, S, d], mask broadcastable to [B, Hq, T, S].
    Returns [B, T, Hq, d] float64 (the attention interface's output layout).
    """
    G = q.shape[1] // k.shape[1]
    kk = k.double().repeat_interleave(G, dim=1)
    vv = v.double().repeat_interleave(G, dim=1)
    s = torch.matmul(q.double(), kk.transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask.double()
    p = torch.softmax(s, dim=-1)
    return torch.matmul(p, vv).transpose(1, 2)


def biased_attention_ref(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, lw: Optional[torch.Tensor],
                         heads_per_batch: Optional[Sequence[Sequence[int]]], scale: float,
                         model_dtype=torch.bfloat16) -> torch.Tensor:
    """Per batch row: build the hook's mask (prefill if q_len > 1, decode otherwise) and run sdpa_ref.

    lw: [B, W] natural-log weights (fp16 as the reference computes them) or None.
    """
    B, Hq, T, d = q.shape
    S = k.shape[2]
    outs = []
    for b in range(B):
        hs = torch.zeros((1, T, 1), dtype=model_dtype)
        pos = torch.arange(S - T, S)[None]
        if T > 1 and S != T:
            # the hook's own mask assumes the queries start at 0; for q_pos0 > 0 build the
            # equivalent causal mask with the offset (what transformers would pass)
            causal = torch.full((T, S), torch.finfo(model_dtype).min, dtype=model_dtype)
            for i in range(T):
                causal[i, :S - T + i + 1] = 0
            am = causal[None, None]
        else:
            am = None
        if lw is not None and heads_per_batch is not None:
            mask = edit_attention_mask(Hq, hs, am, pos, lw[b:b + 1], heads_per_batch[b])
        else:
            mask = edit_attention_mask(Hq, hs, am, pos, torch.zeros((1, 0), dtype=torch.float16), [])
        outs.append(sdpa_ref(q[b:b + 1], k[b:b + 1], v[b:b + 1], mask, scale))
    return torch.cat(outs, 0)


# ---------------------------------------------------------------------------------------------
# hook registration on a transformers model (the CPU hook path: timed CPU baseline + IE oracle)
# ---------------------------------------------------------------------------------------------
def _pre_hook(module, args, kwargs, *, num_heads, lw, head_idx):
    kwargs["attention_mask"] = edit_attention_mask(num_heads, kwargs["hidden_states"], kwargs["attention_mask"],
                                                   kwargs["position_ids"], lw, head_idx)
    return args, kwargs


def _pre_hook_gpt2(module, args, kwargs, *, num_heads, lw, head_idx):
    """GPT-2 adapter: GPT2Attention gets hidden_states POSITIONALLY and lives at
    transformer.h.{l}.attn, so the reference hook cannot run on it; the same mask edit, with S from
    position_ids (cache_position, or T for a cache-less forward, when absent)."""
    hs = args[0] if args else kwargs["hidden_states"]
    T = hs.shape[1]
    pos = kwargs.get("position_ids")
    if pos is None:
        cp = kwargs.get("cache_position")
        pos = cp.view(1, -1) if cp is not None else torch.arange(T).view(1, -1)
    kwargs["attention_mask"] = edit_attention_mask(num_heads, hs, kwargs.get("attention_mask"), pos, lw, head_idx)
    return args, kwargs


def attention_module_name(model, layer: int) -> str:
    """`model.layers.{l}.self_attn` (re_weighting.py:120) or `transformer.h.{l}.attn` (GPT-2)."""
    return (f"transformer.h.{layer}.attn" if getattr(model.config, "model_type", "") == "gpt2"
            else f"model.layers.{layer}.self_attn")


def register_hooks(model, layers_to_heads: dict, lw: torch.Tensor) -> list:
    """re_weighting.py:118-124 / :163-168: one forward-pre-hook per selected layer."""
    H = model.config.num_attention_heads
    hook = _pre_hook_gpt2 if getattr(model.config, "model_type", "") == "gpt2" else _pre_hook
    handles = []
    for layer, heads in layers_to_heads.items():
        mod = model.get_submodule(attention_module_name(model, int(layer)))
        handles.append(mod.register_forward_pre_hook(partial(hook, num_heads=H, lw=lw, head_idx=list(heads)),
                                                     with_kwargs=True))
    return handles


def answer_logit_sum(logits: torch.Tensor, answer_ids: torch.Tensor) -> torch.Tensor:
    """re_weighting.py:160,170: sum of logits[0, -n+k, a_k] (the answer token's own position)."""
    n = answer_ids.shape[0]
    rows = logits[0, -n:]
    return rows[torch.arange(n), answer_ids].sum()


@torch.no_grad()
def answer_logprobs(model, input_ids: torch.Tensor, lw: torch.Tensor, layers_to_heads: dict, n: int) -> torch.Tensor:
    """Hooked forward (re_weighting.py:118-127 hooks, :36-61 mask) -> fp32 log_softmax of token T-n+k at
    row T-n-1+k, k < n (teacher-forced answer log-probabilities under re-weighting)."""
    hs = register_hooks(model, layers_to_heads, lw)
    try:
        lg = model(input_ids=input_ids, attention_mask=torch.ones_like(input_ids), return_dict=True)["logits"]
    finally:
        for x in hs:
            x.remove()
    T = input_ids.shape[1]
    lp = torch.log_softmax(lg[0, T - n - 1:T - 1].float(), dim=-1)
    return lp.gather(1, input_ids[0, T - n:].view(n, 1)).view(n)


@torch.no_grad()
def ie_grid(model, input_ids: torch.Tensor, lw: torch.Tensor, answer_ids: torch.Tensor,
            layers: Optional[Sequence[int]] = None, heads: Optional[Sequence[int]] = None,
            upcast_logits: bool = False) -> np.ndarray:
    """re_weighting.py:152-175: IE[l][h] = sum(ori answer logits) - sum(hooked answer logits)."""
    L = model.config.num_hidden_layers
    H = model.config.num_attention_heads
    layers = range(L) if layers is None else layers
    heads = range(H) if heads is None else heads

    def run():
        lg = model(input_ids=input_ids, attention_mask=torch.ones_like(input_ids), return_dict=True)["logits"]
        return lg.float() if upcast_logits else lg

    ori = answer_logit_sum(run(), answer_ids)
    out = np.zeros((len(layers), len(heads)), dtype=np.float64)
    for a, l in enumerate(layers):
        for c, h in enumerate(heads):
            hs = register_hooks(model, {l: [h]}, lw)
            try:
                cur = answer_logit_sum(run(), answer_ids)
            finally:
                for x in hs:
                    x.remove()
            out[a, c] = float(ori - cur)
    return out


# ---------------------------------------------------------------------------------------------
# ranking (utils/find_best_heads.py:113-150)
# ---------------------------------------------------------------------------------------------
def combine_all(heads_scores: np.ndarray) -> List[Tuple[float, Tuple[int, int]]]:
    """find_best_heads.py:113-132: mean over questions, flat argsort descending."""
    mean = np.asarray(heads_scores, dtype=np.float64).mean(axis=0)
    flat = mean.reshape(-1)
    order = np.argsort(flat)[::-1]
    rows, cols = np.unravel_index(order, mean.shape)
    return [(float(flat[i]), (int(r), int(c))) for i, r, c in zip(order, rows, cols)]


def top_k_heads(sorted_scores, k: int) -> dict:
    """find_best_heads.py:135-150: first k entries grouped by layer (insertion order)."""
    out: dict = {}
    for _, (l, h) in sorted_scores[:k]:
        out.setdefault(l, []).append(h)
    return out
