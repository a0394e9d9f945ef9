"""Score pipeline (RAG_test.py:64-121) against the reference's saved GPT-setting prompts.

Fixture: tests/golden/score_pipeline.json.gz (gen_scores.py) — per NQ question the passage order of the
re-weighting prompt and the passages kept by delete mode, both cut out of the reference's result files.
"""
import gzip
import json
import os

import numpy as np
import pytest

from cram_amd import scores as sc
from cram_amd import spans

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def nq():
    with gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def fx():
    with gzip.open(os.path.join(REPO, "tests", "golden", "score_pipeline.json.gz"), "rt") as f:
        return {r["id"]: r for r in json.load(f)}


def _ctx(rec):
    return rec["ori_fake"] + rec["reranked_dense_ctxs"]


def test_gpt_weighting_order_matches_reference(nq, fx):
    zero_fake = 0
    for rec in nq:
        ctx = _ctx(rec)
        contexts, scores = sc.assemble(rec)
        assert contexts == [ctx[i] for i in fx[rec["id"]]["weighting_order"]], rec["id"]
        s = np.asarray(scores)
        if s.dtype.kind == "i":                                                # all equal: scores + 1
            assert s.tolist() == [1] * 5
        else:
            assert s.dtype == np.float64 and s.min() == 0.0 and s.max() == 1.0
        assert np.all(np.diff(s) >= 0)
        zero_fake += contexts[0] == ctx[0]
    assert zero_fake > 300            # the fake passage is usually the least credible one (-> -inf bias)


def test_gpt_delete_matches_reference(nq, fx):
    for rec in nq:
        ctx = _ctx(rec)
        contexts, scores = sc.assemble(rec, re_weighting=False, delete_false_paras=True)
        assert scores == []
        assert contexts == [ctx[i] for i in fx[rec["id"]]["delete_kept"]], rec["id"]


def test_ideal_scores():
    rec = {"ori_fake": ["f"], "reranked_dense_ctxs": ["a", "b", "c", "d", "e"]}
    contexts, scores = sc.assemble(rec, ideal=True, ideal_score=1)          # run.sh: ideal_score=1
    assert contexts == ["f", "a", "b", "c", "d"] and scores == [0.1, 1.0, 1.0, 1.0, 1.0]
    contexts, scores = sc.assemble(rec, ideal=True, ideal_score=0)
    assert scores[0] == 0.0 and spans.weight_vector(3, [(0, 0), (1, 1), (2, 2)], scores[:3])[0].isinf().sum() == 0


def test_ties_and_all_equal():
    rec = {"ori_fake": ["f"], "reranked_dense_ctxs": ["a", "b", "c", "d"], "ori_fake_truthful_scores": [7],
           "reranked_dense_ctxs_truthful_scores": [9, 7, 3, 9]}
    contexts, scores = sc.assemble(rec)
    assert contexts == ["c", "f", "b", "a", "d"]                               # stable among equal scores
    assert scores == [0.0, 4 / 6, 4 / 6, 1.0, 1.0]
    rec["ori_fake_truthful_scores"], rec["reranked_dense_ctxs_truthful_scores"] = [5], [5, 5, 5, 5]
    contexts, scores = sc.assemble(rec)                                         # max 0 after -min -> +1, ints
    assert contexts == ["f", "a", "b", "c", "d"] and [int(x) for x in scores] == [1] * 5
    assert np.asarray(scores).dtype.kind == "i"
    contexts, scores = sc.assemble(rec, prompt_type="with_contexts_score", re_weighting=False)
    assert [int(x) for x in scores] == [5] * 5


def test_delete_uses_first_equal_passage():
    rec = {"ori_fake": ["x"], "reranked_dense_ctxs": ["y", "x", "z", "w"], "ori_fake_truthful_scores": [1],
           "reranked_dense_ctxs_truthful_scores": [5, 9, 2, 8]}
    contexts, _ = sc.assemble(rec, re_weighting=False, delete_false_paras=True)
    assert contexts == ["y", "w"]                  # both copies of "x" take the first copy's score (1)


def test_relevant_product():
    rec = {"ori_fake": ["f"], "reranked_dense_ctxs": ["a", "b", "c", "d"], "ori_fake_truthful_scores": [2],
           "reranked_dense_ctxs_truthful_scores": [8, 9, 10, 10], "ori_fake_relevant_scores": [10],
           "reranked_dense_ctxs_relevant_scores": [5, 10, 10, 9]}
    contexts, scores = sc.assemble(rec, relevant=True)                         # no -min in relevant mode
    assert contexts == ["f", "a", "b", "d", "c"] and scores == [0.2, 0.4, 0.9, 0.9, 1.0]
