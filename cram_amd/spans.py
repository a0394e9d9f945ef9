"""Prompt construction and the passage -> token-span rule of the reference.

Reference semantics (must be reproduced bit-for-bit; pinned by tests/golden/spans.json.gz):
  * prompt text          utils/prompt.py:4-12 + utils/prompts_templates.py:5-6 ('with_contexts')
  * chat branch          re_weighting.py:64-97 (Llama-3: system "You are a helpful assistant!",
                         special tokens added -> double BOS; Qwen: "... assistant.", no special
                         tokens; other models: raw template with the answer inline)
  * span rule            re_weighting.py:100-110: for passage i the text "Passage-i: <p>\\n" is
                         located with str.find; its token span is [max{t: start_t <= c0},
                         max{t: start_t <= c1}] over the offset-mapping START of every token,
                         c1 = c0 + len - 1 (the trailing newline)
  * weight vector        re_weighting.py:99,111: fp16 ones, each span overwritten with fp16(score_i)
                         in passage order
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

TEMPLATE_WITH_CONTEXTS = ("Given the following information: \n{paras}\nAnswer the following question based on the "
                          "given information or your internal knowledge with one or few words without the source.\n"
                          "Question: {question}\nAnswer: {answer}")
SYSTEM_PROMPTS = {"llama3": "You are a helpful assistant!", "qwen": "You are a helpful assistant."}


def model_family(model_name: str) -> str:
    """The reference branches on substrings of the model name (re_weighting.py:65,80)."""
    if "Llama-3" in model_name:
        return "llama3"
    if "Qwen" in model_name:
        return "qwen"
    return "plain"


def passage_text(i: int, p: str) -> str:
    return f"Passage-{i}: {p}"


def get_prompt(context: Sequence[str], question: str, answer: str = "") -> str:
    paras = "\n".join(passage_text(i, p) for i, p in enumerate(context))
    return TEMPLATE_WITH_CONTEXTS.format(question=question, paras=paras, answer=answer)


def build_prompt(tokenizer, model_name: str, paras: Sequence[str], question: str,
                 answer: str = "") -> Tuple[str, bool]:
    """Returns (text to tokenise, add_special_tokens)."""
    fam = model_family(model_name)
    if fam == "plain":
        return get_prompt(paras, question, answer), True
    msgs = [{"role": "system", "content": SYSTEM_PROMPTS[fam]},
            {"role": "user", "content": get_prompt(paras, question, "")}]
    text = tokenizer.apply_chat_template(msgs, add_generation_prompt=True, tokenize=False)
    if answer != "":
        text = text + answer
    return text, fam == "llama3"


def token_spans(prompt: str, paras: Sequence[str], offsets) -> List[Tuple[int, int]]:
    """Inclusive token span of every passage (vectorised form of the reference's scan)."""
    starts = np.asarray([int(o[0]) for o in offsets], dtype=np.int64)
    idx = np.arange(len(starts))
    spans = []
    for i, p in enumerate(paras):
        text = passage_text(i, p) + "\n"
        c0 = prompt.find(text)
        c1 = c0 + len(text) - 1
        le0 = idx[starts <= c0]
        le1 = idx[starts <= c1]
        if c0 < 0 or le0.size == 0 or le1.size == 0:
            raise ValueError(f"passage {i} is not in the prompt")
        spans.append((int(le0[-1]), int(le1[-1])))
    return spans


def weight_vector(T: int, spans: Sequence[Tuple[int, int]], scores: Sequence[float]) -> torch.Tensor:
    """fp16 [1, T] credibility weights (1 outside passages)."""
    w = torch.ones((1, T), dtype=torch.float16)
    for (t0, t1), s in zip(spans, scores):
        w[0, t0:t1 + 1] = torch.tensor(float(s), dtype=torch.float32).to(torch.float16)
    return w


def _tokenize_batch(tokenizer, texts: Sequence[str], add_special: bool):
    """[(ids int64 [T], token char starts int64 [T])] — the fast tokenizer's Rust batch encoder when the
    tokenizer has one (same ids/offsets as tokenizer(...), re_weighting.py:98), else tokenizer(...)."""
    backend = getattr(tokenizer, "_tokenizer", None)
    if backend is not None and hasattr(backend, "encode_batch"):
        encs = backend.encode_batch(list(texts), add_special_tokens=add_special)
        return [(np.asarray(e.ids, dtype=np.int64), np.asarray(e.offsets, dtype=np.int64).reshape(-1, 2)[:, 0])
                for e in encs]
    out = []
    for t in texts:
        e = tokenizer([t], return_offsets_mapping=True, add_special_tokens=add_special)
        out.append((np.asarray(e["input_ids"][0], dtype=np.int64),
                    np.asarray(e["offset_mapping"][0], dtype=np.int64).reshape(-1, 2)[:, 0]))
    return out


def encode_batch(tokenizer, model_name: str, questions: Sequence[str], paras_list: Sequence[Sequence[str]],
                 scores_list: Sequence[Sequence[float]], answers: Sequence[str] = None):
    """Batched encode(): [(input_ids int64 [T], fp16 weight [1, T], spans)] per prompt.

    One batch tokenizer call, str.find for the passage character ranges, then the native span builder
    (cram_passage_weights in libcram_attn.so) for spans and fp16 weights of every prompt at once.
    """
    from . import _lib
    n = len(questions)
    answers = [""] * n if answers is None else list(answers)
    texts, flags, lo, hi, sc, cu_par = [], [], [], [], [], [0]
    for q, paras, scores, a in zip(questions, paras_list, scores_list, answers):
        if len(scores) < len(paras):
            raise IndexError("fewer scores than passages (the reference raises the same way at re_weighting.py:111)")
        text, add_special = build_prompt(tokenizer, model_name, list(paras), q, a)
        texts.append(text)
        flags.append(add_special)
        for i, p in enumerate(paras):
            para = passage_text(i, p) + "\n"
            c0 = text.find(para)
            lo.append(c0)
            hi.append(c0 + len(para) - 1)
        sc.extend(float(x) for x in scores[:len(paras)])
        cu_par.append(len(lo))
    if len(set(flags)) > 1:
        raise ValueError("mixed special-token settings in one batch")
    toks = _tokenize_batch(tokenizer, texts, flags[0] if flags else True)
    cu_tok = np.zeros(n + 1, dtype=np.int64)
    cu_tok[1:] = np.cumsum([len(ids) for ids, _ in toks])
    starts = np.concatenate([st for _, st in toks]) if n else np.zeros(0, np.int64)
    cu_par = np.asarray(cu_par, dtype=np.int64)
    lo = np.asarray(lo, dtype=np.int64)
    hi = np.asarray(hi, dtype=np.int64)
    sc32 = np.asarray(sc, dtype=np.float64).astype(np.float32)           # score -> fp32 -> fp16 (re_weighting.py:110)
    span_lo = np.empty(len(lo), dtype=np.int32)
    span_hi = np.empty(len(lo), dtype=np.int32)
    w16 = np.empty(int(cu_tok[-1]), dtype=np.float16)
    ptr = lambda a: a.ctypes.data if a.size else None
    rc = _lib.load().cram_passage_weights(n, ptr(cu_tok), ptr(starts), ptr(cu_par), ptr(lo), ptr(hi), ptr(sc32),
                                          ptr(span_lo), ptr(span_hi), ptr(w16))
    if rc != 0:
        raise ValueError("a passage is not in its prompt (re_weighting.py:102-110 fails the same way)")
    out = []
    for b in range(n):
        t0, t1 = int(cu_tok[b]), int(cu_tok[b + 1])
        sp = list(zip(span_lo[cu_par[b]:cu_par[b + 1]].tolist(), span_hi[cu_par[b]:cu_par[b + 1]].tolist()))
        out.append((torch.from_numpy(toks[b][0]), torch.from_numpy(w16[t0:t1].copy()).view(1, -1), sp))
    return out


def encode(tokenizer, model_name: str, question: str, paras: Sequence[str], scores: Sequence[float],
           answer: str = ""):
    """(text, input_ids [1,T] int64, fp16 weight [1,T], spans) for one question, on the host."""
    if len(scores) < len(paras):
        raise IndexError("fewer scores than passages (the reference raises the same way at re_weighting.py:111)")
    text, add_special = build_prompt(tokenizer, model_name, paras, question, answer)
    enc = tokenizer([text], return_tensors="pt", return_offsets_mapping=True, add_special_tokens=add_special)
    spans = token_spans(text, paras, enc["offset_mapping"][0].tolist())
    w = weight_vector(enc["input_ids"].shape[1], spans, scores)
    return text, enc, w, spans
