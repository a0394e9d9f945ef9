"""Known-answer tests on the reference's own fixtures (copied by tests/golden/gen_fixtures.py).

Ranking: datasets/<ds>/<model>/heads_scores.json -> heads_scores_mean.json -> selected_heads.json
(find_best_heads.py:113-150).  Metrics: results*/details rows (eval.py:13-94).
"""
import gzip
import json
import os

import numpy as np
import pytest

from cram_amd import heads as H
from cram_amd import metrics as M
from oracle import hook_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(os.path.join(GOLD, "heads_fixtures.npz")))


KEYS = ["nq__llama3", "nq__qwen", "nq__llama2_13b_chat", "trivia__llama3", "trivia__qwen"]


@pytest.mark.parametrize("key", KEYS)
def test_mean_values_exact(fx, key):
    ranked = H.rank_heads(fx[key + "__scores"])
    vals = np.array([v for v, _ in ranked])
    np.testing.assert_array_equal(vals, fx[key + "__mean_values"])           # max abs diff 0.0


@pytest.mark.parametrize("key", KEYS)
def test_order_matches_up_to_exact_ties(fx, key):
    ranked = H.rank_heads(fx[key + "__scores"])
    lh = np.array([lh for _, lh in ranked])
    ref_lh = fx[key + "__mean_lh"]
    vals = fx[key + "__mean_values"]
    diff = np.nonzero((lh != ref_lh).any(1))[0]
    for i in diff:        # any disagreement must sit inside a group of exactly-equal means
        same = np.nonzero(vals == vals[i])[0]
        assert len(same) > 1, f"rank {i} differs without a tie"
        assert set(map(tuple, lh[same])) == set(map(tuple, ref_lh[same]))


@pytest.mark.parametrize("key", KEYS + ["trivia__llama2_13b_chat"])
def test_selected_heads_top_k(fx, key):
    k = int(fx[key + "__selected_k"][0])
    sel = fx[key + "__selected"]
    if key + "__scores" in fx:
        ranked = H.rank_heads(fx[key + "__scores"])
    else:   # no per-question file: rank from the saved means
        ranked = [(float(v), tuple(map(int, lh))) for v, lh in zip(fx[key + "__mean_values"], fx[key + "__mean_lh"])]
    top = H.top_k(ranked, k)
    got = sorted((l, h) for l, hs in top.items() for h in hs)
    assert got == sorted(map(tuple, sel.tolist()))
    # the oracle restatement agrees as a set too
    if key + "__scores" in fx:
        oref = hook_ref.top_k_heads(hook_ref.combine_all(fx[key + "__scores"]), k)
        assert sorted((l, h) for l, hs in oref.items() for h in hs) == got


def test_top_head_is_30_14(fx):
    v, lh = H.rank_heads(fx["nq__llama3__scores"])[0]
    assert lh == (30, 14) and abs(v - 0.5079) < 1e-4


def test_rank_deterministic_ties():
    a = np.zeros((2, 2, 3))
    a[:, 0, 1] = 1.0
    r = H.rank_heads(a)
    assert r[0][1] == (0, 1)
    assert [lh for _, lh in r[1:]] == [(1, 2), (1, 1), (1, 0), (0, 2), (0, 0)]


def test_file_drivers_roundtrip(tmp_path, fx):
    d = tmp_path / "nq" / "llama3"
    d.mkdir(parents=True)
    (d / "heads_scores.json").write_text(json.dumps(fx["nq__llama3__scores"].tolist()))
    H.casual_tracing_combine_all(str(d))
    sel = H.find_top_k_heads(str(d), 894)
    got = sorted((int(l), h) for l, hs in sel.items() for h in hs)
    assert got == sorted(map(tuple, fx["nq__llama3__selected"].tolist()))


@pytest.fixture(scope="module")
def evalfx():
    with gzip.open(os.path.join(GOLD, "eval_fixtures.json.gz"), "rt", encoding="utf-8") as f:
        return json.load(f)


def test_em_f1_rows(evalfx):
    n = 0
    for blob in evalfx:
        rows = [dict(r) for r in blob["rows"]]
        summary = M.evaluate(rows)
        for r, g in zip(rows, blob["rows"]):
            assert r["Eval"] == g["Eval"]
            assert r["f1_score"] == pytest.approx(g["f1_score"], abs=1e-12)
            n += 1
        lines = blob["accuracy"].splitlines()
        assert lines[0] == f"Accuracy: {summary['accuracy']:.4f}"
        assert lines[1] == f"EM: {summary['em']}/{summary['n']}"
        assert lines[2] == f"F1: {summary['f1']:.4f}"
    assert n == 5000


def test_published_em(evalfx):
    blob = [b for b in evalfx if "ideal_heads894" in b["file"]][0]
    assert M.evaluate([dict(r) for r in blob["rows"]])["accuracy"] == pytest.approx(0.369)


def test_metric_edge_cases():
    assert M.exact_match("", ["x"]) is False
    assert M.exact_match("The Answer!", ["answer"]) is True
    assert M.f1_score("", "") == 1
    assert M.f1_score("a b", "c") == 0


def test_gemm_pin_file_signatures():
    """The pinned GEMM lines use TunableOp's own signature for F.linear (x [M, K] @ w[N, K]^T = TN, m = N, n = M)
    as written by a tuning run (tools/tunable_probe.py), and every pinned shape is a Llama-3-8B projection."""
    from cram_amd import gemm_tune
    assert gemm_tune._signature(6144, 4096, 29184) == "tn_6144_29184_4096_ld_4096_4096_6144"
    sol = gemm_tune.load()
    assert set(sol["solutions"]) <= {"6144x4096", "4096x4096", "28672x4096", "4096x14336"}
    assert {"HIPBLASLT_VERSION", "ROCBLAS_VERSION", "GCN_ARCH_NAME"} <= set(sol["validators"])
    rows = gemm_tune.sweep_rows()
    assert rows[0] == 8192 and rows[-1] == 65536 and all(m % 256 == 0 for m in rows)
