"""IE-sweep drivers and influential-head ranking (utils/find_best_heads.py, same file formats).

  casual_tracing_per_head       find_best_heads.py:13-58   per-question IE grid, resume by skipping
  casual_tracing_per_head_with_position  :61-110          fake passage moved through positions 0..4,
                                                           heads_scores_pos.json rewritten per question (+resume)
  casual_tracing_combine_all    :113-132                   mean over questions, ranking
  find_top_k_heads              :135-150                   top-k -> {layer: [heads]}

Ranking tie-break: the reference uses np.argsort(flat)[::-1] (quicksort, so the
order of exactly-equal means depends on the numpy version).  Here the order is
fixed: value descending, then flat index (layer*H + head) DESCENDING — which is
what a stable ascending sort reversed yields, and what the reference's
fixtures show for the tied pairs we checked (tests/test_ranking.py).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Sequence, Tuple

import numpy as np


def rank_heads(heads_scores) -> List[Tuple[float, Tuple[int, int]]]:
    """[Nq, L, H] (or [L, H]) IE -> [(mean IE, (layer, head))] sorted, deterministic tie-break."""
    a = np.asarray(heads_scores, dtype=np.float64)
    mean = a.mean(axis=0) if a.ndim == 3 else a
    flat = mean.reshape(-1)
    order = np.argsort(flat, kind="stable")[::-1]
    L, H = mean.shape
    return [(float(flat[i]), (int(i // H), int(i % H))) for i in order]


def top_k(ranked: Sequence[Tuple[float, Tuple[int, int]]], k: int) -> Dict[int, List[int]]:
    out: Dict[int, List[int]] = {}
    for _, (l, h) in ranked[:k]:
        out.setdefault(l, []).append(h)
    return out


def casual_tracing_combine_all(input_path: str) -> list:
    with open(os.path.join(input_path, "heads_scores.json"), encoding="utf-8") as f:
        data = json.load(f)
    ranked = rank_heads(data)
    with open(os.path.join(input_path, "heads_scores_mean.json"), "w", encoding="utf-8") as f:
        json.dump([(v, list(lh)) for v, lh in ranked], f, ensure_ascii=False, indent=4)
    return ranked


def find_top_k_heads(input_path: str, topk: int = 10) -> Dict[int, List[int]]:
    with open(os.path.join(input_path, "heads_scores_mean.json"), encoding="utf-8") as f:
        data = json.load(f)
    sel: Dict[int, List[int]] = {}
    for _, (l, h) in data[:topk]:
        sel.setdefault(l, []).append(h)
    with open(os.path.join(input_path, "selected_heads.json"), "w", encoding="utf-8") as f:
        json.dump(sel, f, ensure_ascii=False, indent=4)
    return sel


def sweep_contexts(sample: dict, contexts_type=("ori_fake", "reranked_dense"), topk: int = 4):
    """find_best_heads.py:41-48: contexts and the sweep scores [0] + [1]*4."""
    contexts, scores = [], []
    if "ori_fake" in contexts_type:
        contexts.extend(sample["ori_fake"])
        scores.extend([0])
    if "reranked_dense" in contexts_type:
        contexts.extend(sample["reranked_dense_ctxs"][:topk])
        scores.extend([1, 1, 1, 1])
    return contexts, scores


def casual_tracing_per_head(data: list, model, output_file: str, contexts_type=("ori_fake", "reranked_dense"),
                            topk: int = 4) -> list:
    """Per-question IE grids appended to output_file, resuming after the questions already present."""
    done = []
    if os.path.exists(output_file):
        with open(output_file, encoding="utf-8") as f:
            done = json.load(f)
    for idx, sample in enumerate(data):
        if idx < len(done):
            continue
        ctx, sc = sweep_contexts(sample, contexts_type, topk)
        wrong = sample.get("wrong answer", sample.get("wrong_answer"))
        done.append(model.cal_logits(question=sample["question"], paras=ctx, scores=sc, wrong_answer=wrong))
        os.makedirs(os.path.dirname(os.path.abspath(output_file)), exist_ok=True)
        tmp = output_file + ".tmp"
        with open(tmp, "w", encoding="utf-8") as f:
            json.dump(done, f, ensure_ascii=False, indent=4)
        os.replace(tmp, output_file)
    return done


def casual_tracing_per_head_sharded(data: list, model, output_file: str, shard_dir: str,
                                    contexts_type=("ori_fake", "reranked_dense"), topk: int = 4, group=None) -> list:
    """casual_tracing_per_head (find_best_heads.py:13-58) over one process per GPU: the (question, layer) units of
    all questions are sharded over the ranks (cram_amd.dist.plan), every rank checkpoints its finished units in
    shard_dir/rank{r}.jsonl (a restarted run of any world size skips them), one all-gather assembles [Nq, L, H]
    and rank 0 writes heads_scores.json in the reference's format.  `model` is a Find_Best_Heads."""
    import torch.distributed as tdist
    qs, ps, ss, ws = [], [], [], []
    for sample in data:
        ctx, sc = sweep_contexts(sample, contexts_type, topk)
        qs.append(sample["question"])
        ps.append(ctx)
        ss.append(sc)
        ws.append(sample.get("wrong answer", sample.get("wrong_answer")))
    ie = model.cal_logits_batch(qs, ps, ss, ws, shard_dir=shard_dir, group=group)
    res = ie.double().cpu().numpy().tolist()
    if not tdist.is_initialized() or tdist.get_rank(group) == 0:
        os.makedirs(os.path.dirname(os.path.abspath(output_file)), exist_ok=True)
        tmp = output_file + ".tmp"
        with open(tmp, "w", encoding="utf-8") as f:
            json.dump(res, f, ensure_ascii=False, indent=4)
        os.replace(tmp, output_file)
    return res


def position_contexts(sample: dict, position: int, contexts_type=("ori_fake", "reranked_dense"), topk: int = 4):
    """find_best_heads.py:83-99: the retrieved passages before `position`, then the fake passage(s), then the rest.

    Quirk kept: every "ori_fake" passage is inserted but ONE score 0 is appended (:93-94), as in the plain sweep;
    the retrieved passages always get [1] * position and [1] * (4 - position) (:89, :99), whatever topk is."""
    docs = sample["reranked_dense_ctxs"][:topk]
    contexts, scores = [], []
    if "reranked_dense" in contexts_type:
        contexts.extend(docs[:position])
        scores.extend([1] * position)
    if "ori_fake" in contexts_type:
        contexts.extend(sample["ori_fake"])
        scores.append(0)
    if "reranked_dense" in contexts_type:
        contexts.extend(docs[position:])
        scores.extend([1] * (4 - position))
    return contexts, scores


def casual_tracing_per_head_with_position(data: list, model, output_file: str = None,
                                          contexts_type=("ori_fake", "reranked_dense"), topk: int = 4,
                                          resume: bool = True) -> list:
    """find_best_heads.py:61-110: per question, the IE grid with the fake passage at positions 0..4 among the
    retrieved ones -> [Nq][5][L][H].

    Like the reference, the whole list is rewritten to `output_file` (heads_scores_pos.json) after every
    question (:105-110).  Added: with resume=True the questions already in the file are skipped (the reference
    restarts from [] on every run, :76, losing 5 x L x H units per finished question when a run dies); a
    question is written only once all five positions are done, so a partial question is recomputed."""
    done = []
    if output_file and resume and os.path.exists(output_file):
        with open(output_file, encoding="utf-8") as f:
            done = json.load(f)
    for idx, sample in enumerate(data):
        if idx < len(done):
            continue
        wrong = sample.get("wrong answer", sample.get("wrong_answer"))
        per_pos = []
        for position in range(5):
            ctx, sc = position_contexts(sample, position, contexts_type, topk)
            per_pos.append(model.cal_logits(question=sample["question"], paras=ctx, scores=sc, wrong_answer=wrong))
        done.append(per_pos)
        if output_file:
            os.makedirs(os.path.dirname(os.path.abspath(output_file)), exist_ok=True)
            tmp = output_file + ".tmp"
            with open(tmp, "w", encoding="utf-8") as f:
                json.dump(done, f, ensure_ascii=False, indent=4)
            os.replace(tmp, output_file)          # a kill mid-write leaves the previous complete file
    return done
