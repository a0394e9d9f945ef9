"""CPU known-answer tests against vectors produced by the reference itself (tests/golden/gen_golden.py).

G1 spans/weights, G2 hook masks: bit-exact for the product (cram_amd.spans,
cram_amd.bias, Re_Weighting_Strategy.edit_attention_mask) and for the oracle.
"""
import gzip
import json
import os

import numpy as np
import pytest
import torch

from cram_amd import spans as S
from cram_amd.bias import bias_from_weight, head_enable
from oracle import hook_ref
from tests import tiny_models as tm

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def span_rows():
    with gzip.open(os.path.join(GOLD, "spans.json.gz"), "rt", encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def toks(tmp_path_factory):
    """Tokenizers loaded from saved tiny-model dirs, exactly as the reference (and the product) load them."""
    from transformers import AutoTokenizer
    root = str(tmp_path_factory.mktemp("tiny"))
    return {k: AutoTokenizer.from_pretrained(tm.save_model(k, root)) for k in ("llama3", "qwen2")}


NAMES = {"llama3": "/x/Llama-3-tiny", "qwen2": "/x/Qwen2-tiny"}


def test_spans_product_bit_exact(span_rows, toks):
    assert len(span_rows) == 96
    for r in span_rows:
        _, enc, w, _ = S.encode(toks[r["kind"]], NAMES[r["kind"]], r["question"], r["paras"], r["scores"], r["answer"])
        assert enc["input_ids"][0].tolist() == r["input_ids"], (r["kind"], r["ds"], r["idx"], r["variant"])
        assert w[0].float().tolist() == r["weight"], (r["kind"], r["ds"], r["idx"], r["variant"])


def test_spans_oracle_bit_exact(span_rows, toks):
    for r in span_rows[::5]:
        tok = toks[r["kind"]]
        text, add = hook_ref.chat_prompt(tok, NAMES[r["kind"]], r["paras"], r["question"], r["answer"])
        enc = tok([text], return_offsets_mapping=True, add_special_tokens=add)
        sp = hook_ref.token_spans(text, r["paras"], enc["offset_mapping"][0])
        w = hook_ref.weight_vector(len(enc["input_ids"][0]), sp, r["scores"])
        assert enc["input_ids"][0] == r["input_ids"]
        assert w[0].float().tolist() == r["weight"]


def test_llama3_double_bos_and_qwen_no_bos(span_rows, toks):
    l3 = [r for r in span_rows if r["kind"] == "llama3"][0]
    bos = toks["llama3"].bos_token_id
    assert l3["input_ids"][:2] == [bos, bos]
    qw = [r for r in span_rows if r["kind"] == "qwen2"][0]
    assert qw["input_ids"][0] == toks["qwen2"].convert_tokens_to_ids("<|im_start|>")


def test_sweep_scores_give_minus_inf_bias(span_rows):
    r = [x for x in span_rows if x["variant"] == "sweep"][0]
    w = torch.tensor(r["weight"], dtype=torch.float16)[None]
    b = bias_from_weight(w, torch.bfloat16)[0]
    assert torch.isinf(b).sum() > 10 and (b[torch.isfinite(b)] == 0).all()
    r = [x for x in span_rows if x["variant"] == "ideal"][0]
    b = bias_from_weight(torch.tensor(r["weight"], dtype=torch.float16)[None], torch.bfloat16)[0]
    vals = set(b.tolist())
    assert vals == {0.0, -2.296875}, vals    # bf16(log_fp16(fp16(0.1)))


@pytest.fixture(scope="module")
def masks():
    return dict(np.load(os.path.join(GOLD, "masks.npz")))


def _dense_from_descriptor(bias_row, en, T, S_, dt, q_pos0, given=None):
    """Rebuild the dense mask from the O(S) descriptor (what the kernels add to the scores)."""
    H = en.shape[0]
    mn = torch.finfo(dt).min
    if given is None:
        m = torch.zeros((1, 1, T, S_), dtype=dt)
        if T > 1:
            m = torch.triu(torch.full((T, S_), mn, dtype=dt), 1)[None, None]
    else:
        m = given.clone()
    m = m.repeat(1, H, 1, 1)
    W = bias_row.shape[0]
    for h in range(H):
        if en[h]:
            sub = m[0, h, :, :W]
            allowed = sub == 0
            sub[allowed] = bias_row.to(dt)[None].expand(T, W)[allowed]
    return m


@pytest.mark.parametrize("dt_name,dt", [("bf16", torch.bfloat16), ("fp16", torch.float16), ("fp32", torch.float32)])
@pytest.mark.parametrize("heads_name,heads", [("h1", [1]), ("hall", [0, 1, 2, 3]), ("h02", [0, 2])])
def test_hook_masks(masks, dt_name, dt, heads_name, heads):
    lw = torch.from_numpy(masks["lw"]).to(torch.float16)
    T = 30
    # oracle
    m = hook_ref.edit_attention_mask(4, torch.zeros((1, T, 8), dtype=dt), None, torch.arange(T)[None], lw, heads)
    np.testing.assert_array_equal(m.float().numpy(), masks[f"prefill_{dt_name}_{heads_name}"])
    m = hook_ref.edit_attention_mask(4, torch.zeros((1, 1, 8), dtype=dt), None, torch.tensor([[T + 5]]), lw, heads)
    np.testing.assert_array_equal(m.float().numpy(), masks[f"decode_{dt_name}_{heads_name}"])
    # product utility (Re_Weighting_Strategy.edit_attention_mask)
    from cram_amd.re_weighting import Re_Weighting_Strategy
    obj = object.__new__(Re_Weighting_Strategy)
    obj.model_num_attention_heads = 4
    given = torch.triu(torch.full((T, T), torch.finfo(dt).min, dtype=dt), 1)[None, None]
    given[..., :, 2] = torch.finfo(dt).min
    for key, kw in (("prefill", {"hidden_states": torch.zeros((1, T, 8), dtype=dt), "attention_mask": None,
                                 "position_ids": torch.arange(T)[None]}),
                    ("decode", {"hidden_states": torch.zeros((1, 1, 8), dtype=dt), "attention_mask": None,
                                "position_ids": torch.tensor([[T + 5]])}),
                    ("given", {"hidden_states": torch.zeros((1, T, 8), dtype=dt), "attention_mask": given,
                               "position_ids": torch.arange(T)[None]})):
        _, out = obj.edit_attention_mask(None, (), dict(kw), lw, heads)
        np.testing.assert_array_equal(out["attention_mask"].float().numpy(), masks[f"{key}_{dt_name}_{heads_name}"])
    # the O(S) descriptor the kernels consume reproduces the dense mask exactly
    en = head_enable({0: heads}, 1, 4)[0]
    b = lw[0].to(dt).float()     # bias_from_weight(w, dt): dtype(log_fp16(w)) widened to fp32
    np.testing.assert_array_equal(_dense_from_descriptor(b, en, T, T, dt, 0).float().numpy(),
                                  masks[f"prefill_{dt_name}_{heads_name}"])
    np.testing.assert_array_equal(_dense_from_descriptor(b, en, 1, T + 6, dt, T + 5).float().numpy(),
                                  masks[f"decode_{dt_name}_{heads_name}"])
    np.testing.assert_array_equal(_dense_from_descriptor(b, en, T, T, dt, 0, given).float().numpy(),
                                  masks[f"given_{dt_name}_{heads_name}"])


def test_bias_from_weight_matches_hook_value():
    w = torch.tensor([[1.0, 0.1, 0.0, 0.5, 0.25]], dtype=torch.float16)
    b = bias_from_weight(w, torch.bfloat16)
    ref = torch.log(w).to(torch.bfloat16).float()
    assert torch.equal(b, ref)
    assert b[0, 1].item() == -2.296875 and b[0, 2].item() == float("-inf") and b[0, 0].item() == 0.0


def test_head_enable_string_keys():
    en = head_enable({"3": [1, 2], "0": [0]}, 4, 4)
    assert en.sum() == 3 and en[3, 1] == 1 and en[3, 2] == 1 and en[0, 0] == 1
    with pytest.raises(ValueError):
        head_enable({"9": [0]}, 4, 4)


def test_missing_passage_raises(toks):
    with pytest.raises(ValueError):
        S.token_spans("no passages here", ["abc"], [(0, 2), (3, 5)])
    with pytest.raises(IndexError):
        S.encode(toks["llama3"], NAMES["llama3"], "q?", ["a", "b"], [1.0])


def test_spans_native_batch_bit_exact(span_rows, toks):
    """encode_batch (batch tokenizer + cram_passage_weights in libcram_attn.so) vs the reference's vectors."""
    for kind in ("llama3", "qwen2"):
        rows = [r for r in span_rows if r["kind"] == kind]
        out = S.encode_batch(toks[kind], NAMES[kind], [r["question"] for r in rows], [r["paras"] for r in rows],
                             [r["scores"] for r in rows], [r["answer"] for r in rows])
        for r, (ids, w, sp) in zip(rows, out):
            assert ids.tolist() == r["input_ids"], (kind, r["ds"], r["idx"], r["variant"])
            assert w[0].float().tolist() == r["weight"], (kind, r["ds"], r["idx"], r["variant"])


def test_native_span_rule_edge_cases():
    """cram_passage_weights directly: non-monotone offsets, overlap order, fp16 rounding, errors."""
    from cram_amd import _lib
    L = _lib.load()

    def run(starts, lo, hi, sc):
        cu_tok = np.array([0, len(starts)], np.int64)
        cu_par = np.array([0, len(lo)], np.int64)
        st = np.asarray(starts, np.int64)
        lo_, hi_ = np.asarray(lo, np.int64), np.asarray(hi, np.int64)
        s = np.asarray(sc, np.float32)
        a, e = np.zeros(len(lo), np.int32), np.zeros(len(lo), np.int32)
        w = np.zeros(len(starts), np.float16)
        rc = L.cram_passage_weights(1, cu_tok.ctypes.data, st.ctypes.data, cu_par.ctypes.data, lo_.ctypes.data,
                                    hi_.ctypes.data, s.ctypes.data, a.ctypes.data, e.ctypes.data, w.ctypes.data)
        return rc, list(zip(a.tolist(), e.tolist())), w

    # the reference's scan takes the LAST token whose start <= c, also when offsets are not monotone
    starts = [0, 0, 5, 9, 0, 14, 20]
    rc, sp, w = run(starts, [9], [19], [0.1])
    ref = [max(t for t, x in enumerate(starts) if x <= c) for c in (9, 19)]
    assert rc == 0 and sp == [tuple(ref)] == [(4, 5)]
    assert w.tolist() == [1, 1, 1, 1, np.float16(0.1), np.float16(0.1), 1]
    # overlapping spans: later passage wins; fp32 -> fp16 rounding of the score
    rc, sp, w = run([0, 3, 6, 9, 12], [3, 6], [8, 13], [0.3, 1 / 3])
    assert rc == 0 and sp == [(1, 2), (2, 4)]
    assert w.view(np.uint16).tolist()[1:] == [np.float16(0.3).view(np.uint16), *[np.float16(np.float32(1 / 3))
                                                                                  .view(np.uint16)] * 3]
    assert run([0, 3], [-1], [5], [1.0])[0] == -1          # passage not found
    assert run([4, 8], [2], [9], [1.0])[0] == -1           # precedes every token


@pytest.mark.parametrize("fixture", ["logprobs.json.gz", "llama2_logprobs.json.gz"])
def test_oracle_answer_logprobs_bit_exact(fixture, tmp_path_factory):
    """G6: the oracle's hook restatement on the same transformers model reproduces the reference hook's
    re-weighted answer log-probabilities exactly (bf16 Llama-3 / Qwen2, fp16 Llama-2 and their fp32 copies;
    the Llama-2 rows also pin the raw-template prompt branch the reference's default model takes)."""
    from transformers import AutoModelForCausalLM, AutoTokenizer
    with gzip.open(os.path.join(GOLD, fixture), "rt", encoding="utf-8") as f:
        logprob_rows = json.load(f)
    root = str(tmp_path_factory.mktemp("tinylp"))
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        nq = json.load(f)
    models, toks_ = {}, {}
    for r in logprob_rows:
        key = (r["kind"], r["fp32"])
        if key not in models:
            path = tm.save_model(r["kind"], root, fp32=r["fp32"])
            models[key] = AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval()
            toks_[key] = (AutoTokenizer.from_pretrained(path), path)
        tok, path = toks_[key]
        rec = nq[r["idx"]]
        scores = [0.1, 1, 1, 1, 1] if r["scores"] == "ideal" else [0, 1, 1, 1, 1]
        _, enc, w, _ = S.encode(tok, path, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"], scores,
                                rec["wrong_answer"])
        assert enc["input_ids"][0].tolist() == r["ids"]
        heads = {int(k): v for k, v in r["layers_to_heads"].items()}
        lp = hook_ref.answer_logprobs(models[key], torch.tensor([r["ids"]]), hook_ref.log_weight(w), heads, r["n"])
        assert lp.tolist() == r["logprobs"], (r["kind"], r["fp32"], r["idx"], r["scores"], r["heads"])
