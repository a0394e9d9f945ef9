"""Per-question context/score assembly — the step between a dataset record and Re_Weighting_Strategy.

Restates RAG_test.py:64-107 (the loop body of RAG_gen before run_RAG): which passages go into the
prompt, which credibility score each one gets, the normalisation and the stable re-ordering by score.
The output (contexts, scores) is what run_RAG_with_attention_weighting / run_RAG_batch take.

Numeric details reproduced on purpose:
- scores are built from int(...) of the dataset's truthful / relevant scores (RAG_test.py:91-95);
- GPT setting (not ideal, not relevant): scores -= min(scores) (:95-96), so the least credible
  passage gets 0 -> a -inf bias (re_weighting.py:122);
- scores / max(scores) in float64, or scores + 1 (still ints) when max == 0 (:97-100);
- Python's stable sorted() on the score alone, so equal scores keep their original order (:101-105);
- with_contexts_score / with_contexts_cag prompts sort by the raw int scores (:106-115);
- delete mode keeps passages with score > 3 in original order, looking each passage up by its
  FIRST equal string (contexts.index, :116-121).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

DEFAULT_CONTEXTS = ("ori_fake", "reranked_dense")


def _raw_scores(sample: dict, contexts_type: Sequence[str], ideal: bool, ideal_score: float, relevant: bool,
                topk: int, fake_num: int, need_scores: bool):
    contexts: List[str] = []
    truthful: list = []
    relevant_s: list = []
    if "ori_fake" in contexts_type:                                         # RAG_test.py:69-78
        contexts.extend(sample["ori_fake"][:fake_num])
        if need_scores:
            if ideal:
                truthful.extend([ideal_score] * fake_num)
                relevant_s.extend([10] * fake_num)
            else:
                truthful.extend(sample["ori_fake_truthful_scores"][:fake_num])
                if relevant:
                    relevant_s.extend(sample["ori_fake_relevant_scores"][:fake_num])
    if "reranked_dense" in contexts_type:                                   # RAG_test.py:79-88
        contexts.extend(sample["reranked_dense_ctxs"][:topk])
        if need_scores:
            if ideal:
                truthful.extend([10] * topk)
                relevant_s.extend([10] * topk)
            else:
                truthful.extend(sample["reranked_dense_ctxs_truthful_scores"][:topk])
                if relevant:
                    relevant_s.extend(sample["reranked_dense_ctxs_relevant_scores"][:topk])
    return contexts, truthful, relevant_s


def _int_scores(truthful, relevant_s, relevant: bool) -> np.ndarray:
    s = np.array([int(x) for x in truthful])
    if relevant:
        s = s * np.array([int(x) for x in relevant_s])
    return s


def _stable_sort(scores, contexts) -> Tuple[list, list]:
    pairs = sorted(zip(scores, contexts), key=lambda x: x[0])             # stable on the score only
    if not pairs:
        return [], []
    s, c = zip(*pairs)
    return list(s), list(c)


def assemble(sample: dict, *, prompt_type: str = "with_contexts", contexts_type: Sequence[str] = DEFAULT_CONTEXTS,
             re_weighting: bool = True, delete_false_paras: bool = False, ideal: bool = False,
             ideal_score: float = 0, relevant: bool = False, topk: int = 4,
             fake_num: int = 1) -> Tuple[List[str], list]:
    """(contexts, scores) for one dataset record, as RAG_test.py:64-121 hands them to run_RAG.

    `ideal`/`ideal_score` are whether_ideal_scores / ideal_score (run.sh uses ideal_score=1 -> the fake
    passage gets 0.1); `relevant` is whether_relevant.  Without re-weighting, score prompts or delete
    mode the reference passes scores=[] (:65).
    """
    scored_type = prompt_type in ("with_contexts_score", "with_contexts_cag")
    need = re_weighting or delete_false_paras or scored_type
    contexts, truthful, relevant_s = _raw_scores(sample, contexts_type, ideal, ideal_score, relevant, topk,
                                                 fake_num, need)
    scores: list = []
    if re_weighting and not delete_false_paras:                            # RAG_test.py:89-105
        s = _int_scores(truthful, relevant_s, relevant)
        if not relevant and not ideal:
            s -= np.min(s)
        s = s / np.max(s) if np.max(s) != 0 else s + 1
        scores, contexts = _stable_sort(s, contexts)
    if scored_type:                                                        # RAG_test.py:106-115
        s = _int_scores(truthful, relevant_s, relevant)
        scores, contexts = _stable_sort(s, contexts)
    if delete_false_paras:                                                 # RAG_test.py:116-121
        s = _int_scores(truthful, relevant_s, relevant)
        contexts = [c for c in contexts if s[contexts.index(c)] > 3]
    return contexts, scores

