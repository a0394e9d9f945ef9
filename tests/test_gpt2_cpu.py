"""GPT-2 (MHA, head_dim 64, transformer.h.{l}.attn) on the host.

The reference's hook cannot address GPT-2 (re_weighting.py:120 names model.layers.{l}.self_attn and reads
hidden_states from kwargs, which GPT2Block passes positionally), so GPT-2 results are pinned only through
the mask semantics the oracle shares with the other families (G2): parity here is oracle-vs-product, the
oracle's GPT-2 adapter itself is "parity unpinned" against the reference.
"""
import gzip
import json
import os

import pytest
import torch

from cram_amd import spans
from oracle import hook_ref
from tests import cpu_ops
from tests import tiny_models as tm


@pytest.fixture(scope="module")
def gpt2(tmp_path_factory):
    from transformers import AutoModelForCausalLM, AutoTokenizer
    root = str(tmp_path_factory.mktemp("gpt2"))
    path = tm.save_model("gpt2", root)
    return path, AutoTokenizer.from_pretrained(path), AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval()


@pytest.fixture(scope="module")
def nq():
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        return json.load(f)


def test_gpt2_plain_template_and_spans(gpt2, nq):
    path, tok, _ = gpt2
    rec = nq[0]
    paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
    text, enc, w, sp = spans.encode(tok, path, rec["question"], paras, [0.1, 1, 1, 1, 1], rec["wrong_answer"])
    assert spans.model_family(path) == "plain"
    assert text == hook_ref.get_prompt(paras, rec["question"], rec["wrong_answer"])   # raw template + answer
    assert len(sp) == 5 and all(a <= b for a, b in sp)
    assert (w[0, sp[0][0]:sp[0][1] + 1] == torch.tensor(0.1, dtype=torch.float16)).all()


def test_gpt2_dropin_matches_hooked_oracle(gpt2, nq):
    """cram_hip attention (CPU stand-in kernels) + CredibilityBias == the oracle's hooked sdpa GPT-2."""
    from transformers import AutoModelForCausalLM
    from cram_amd import attention as A
    from cram_amd.bias import CredibilityBias
    path, tok, model = gpt2
    A.register()
    m2 = AutoModelForCausalLM.from_pretrained(path, dtype="auto", attn_implementation=A.IMPL_NAME).eval()
    assert [l for l, _ in A.attention_modules(m2)] == [0, 1, 2]
    rec = nq[1]
    _, enc, w, _ = spans.encode(tok, path, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                [0, 1, 1, 1, 1], rec["wrong_answer"])
    ids = enc["input_ids"]
    n = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"].shape[1] - 1
    T = ids.shape[1]
    for heads in ({0: [1], 2: [0, 3]}, {l: list(range(4)) for l in range(3)}):
        ref = hook_ref.answer_logprobs(model, ids, hook_ref.log_weight(w), heads, n)
        plain = hook_ref.answer_logprobs(model, ids, hook_ref.log_weight(w), {}, n)
        cb = CredibilityBias.build([w], heads, 3, 4, "cpu")
        with cpu_ops.patched_ops(), torch.no_grad(), A.reweighting(m2, cb):
            lg = m2(input_ids=ids).logits
        lp = torch.log_softmax(lg[0, T - n - 1:T - 1].float(), -1).gather(1, ids[0, T - n:].view(n, 1)).view(n)
        assert (lp - ref).abs().max() < 0.05
        assert (ref - plain).abs().max() > 2 * (lp - ref).abs().max()      # the re-weighting is what is measured


def test_gpt2_hooked_generate_runs(gpt2, nq):
    """The adapter also covers cached decode steps (position_ids give S)."""
    path, tok, model = gpt2
    rec = nq[2]
    _, enc, w, _ = spans.encode(tok, path, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                [0.1, 1, 1, 1, 1])
    hs = hook_ref.register_hooks(model, {1: [2]}, hook_ref.log_weight(w))
    try:
        with torch.no_grad():
            out = model.generate(input_ids=enc["input_ids"], attention_mask=enc["attention_mask"], do_sample=False,
                                 max_new_tokens=4)
    finally:
        for h in hs:
            h.remove()
    assert out.shape[1] == enc["input_ids"].shape[1] + 4
