"""casual_tracing_per_head_with_position (find_best_heads.py:61-110) on the CPU: contexts per position, the
heads_scores_pos.json file rewritten after every question, resume after a killed run, and each position's IE
equal to the plain sweep on the passages reordered by hand.  The sweep runs on the tiny Qwen2 model with the
test-only CPU stand-ins of the kernels (tests/cpu_ops.py)."""
import gzip
import json
import os

import numpy as np
import pytest
import torch

from cram_amd import heads as H
from cram_amd import spans, sweep
from tests import cpu_ops
from tests import tiny_models as tm


@pytest.fixture(scope="module")
def nq():
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        return json.load(f)


def test_position_contexts_follow_the_reference(nq):
    rec = nq[0]
    docs, fake = rec["reranked_dense_ctxs"][:4], rec["ori_fake"]
    for pos in range(5):
        ctx, sc = H.position_contexts(rec, pos)
        assert ctx == docs[:pos] + list(fake) + docs[pos:]
        assert sc == [1] * pos + [0] + [1] * (4 - pos)
    ctx, sc = H.position_contexts(rec, 2, contexts_type=("reranked_dense",))
    assert ctx == docs and sc == [1, 1, 1, 1]
    ctx, sc = H.position_contexts(rec, 3, contexts_type=("ori_fake",))
    assert ctx == list(fake) and sc == [0]
    # quirk (find_best_heads.py:93-94): every fake passage is inserted, one score appended
    two = dict(rec, ori_fake=["fake one", "fake two"])
    ctx, sc = H.position_contexts(two, 1)
    assert ctx == docs[:1] + ["fake one", "fake two"] + docs[1:] and len(sc) == 5


class _SweepModel:
    """cal_logits through the head-batched sweep (what Find_Best_Heads.cal_logits runs), recording its calls."""

    def __init__(self, path, fail_at=None):
        from transformers import AutoModelForCausalLM, AutoTokenizer
        from cram_amd.engine import CrAMEngine
        self.path = path
        self.tok = AutoTokenizer.from_pretrained(path)
        self.eng = CrAMEngine.from_hf(AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval())
        self.calls = []
        self.fail_at = fail_at

    def cal_logits(self, question="", paras=(), scores=(), right_answer="", wrong_answer="my name is"):
        if self.fail_at is not None and len(self.calls) == self.fail_at:
            raise KeyboardInterrupt("simulated kill")
        self.calls.append((question, list(paras), list(scores)))
        _, enc, w, _ = spans.encode(self.tok, self.path, question, list(paras), list(scores), wrong_answer)
        ans = self.tok([wrong_answer], return_tensors="pt")["input_ids"][0, 1:]
        with cpu_ops.patched_ops():
            ie = sweep.ie_question(self.eng, enc["input_ids"][0], w[0], ans)
        return ie.double().numpy().tolist()


def test_position_sweep_file_resume_and_values(tmp_path, nq):
    path = tm.save_model("qwen2", str(tmp_path))
    data = nq[:2]
    out = str(tmp_path / "nq" / "qwen" / "heads_scores_pos.json")
    # a run killed during question 1 (after its 2nd position): question 0 is on file, complete
    m1 = _SweepModel(path, fail_at=7)
    with pytest.raises(KeyboardInterrupt):
        H.casual_tracing_per_head_with_position(data, m1, output_file=out)
    saved = json.load(open(out))
    assert len(saved) == 1 and len(saved[0]) == 5
    # resume: question 0 is not recomputed, question 1 is (all five positions)
    m2 = _SweepModel(path)
    res = H.casual_tracing_per_head_with_position(data, m2, output_file=out)
    assert [c[0] for c in m2.calls] == [data[1]["question"]] * 5
    assert json.load(open(out)) == res and len(res) == 2
    L, Hh = m2.eng.spec.num_layers, m2.eng.spec.num_heads
    assert np.asarray(res).shape == (2, 5, L, Hh)
    # every position equals the sweep on the passages reordered by hand
    for qi, rec in enumerate(data):
        docs = rec["reranked_dense_ctxs"][:4]
        for pos in (0, 2, 4):
            paras = docs[:pos] + rec["ori_fake"] + docs[pos:]
            scores = [1] * pos + [0] + [1] * (4 - pos)
            _, enc, w, _ = spans.encode(m2.tok, path, rec["question"], paras, scores, rec["wrong_answer"])
            ans = m2.tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
            with cpu_ops.patched_ops():
                ref = sweep.ie_question(m2.eng, enc["input_ids"][0], w[0], ans).double().numpy()
            np.testing.assert_array_equal(np.asarray(res[qi][pos]), ref)
    # the fake passage's position changes the IE (the five grids are not copies of one another)
    assert not np.array_equal(np.asarray(res[0][0]), np.asarray(res[0][4]))
    # resume=False restarts from an empty list, as the reference does (find_best_heads.py:76)
    m3 = _SweepModel(path)
    H.casual_tracing_per_head_with_position(data[:1], m3, output_file=out, resume=False)
    assert len(m3.calls) == 5 and len(json.load(open(out))) == 1
