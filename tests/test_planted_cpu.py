"""The planted-IE construction (tests/planted.py) on a tiny Llama-architecture model, float32 truth on the CPU.

Checks the design before it is used at the Llama-3-8B shape (tests/test_topk_identity_gpu.py): the first-order
calibration lands every planted head's IE (re_weighting.py:152-175, as tests/fp32_llama.py computes it) on its
target, the random heads stay near 0, and the mean-IE ranking (find_best_heads.py:113-150, cram_amd.heads.rank_heads)
has exactly the designed top-k sets at the designed boundaries, with gaps far above the bf16 noise level (~0.1).
"""
import gzip
import json
import os

import numpy as np
import torch

from cram_amd import heads as Hd
from cram_amd import spans
from cram_amd.engine import CrAMEngine, ModelSpec
from tests import planted
from tests.fp32_llama import Fp32Llama

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TIERS = ((3, 16.0, 12.0), (5, 8.0, 6.0), (4, 4.0, 3.0))


def _questions(tok, idx):
    data = json.load(gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8"))
    out = []
    for i in idx:
        rec = data[i]
        _, enc, w, _ = spans.encode(tok, "Meta-Llama-3-8B-Instruct", rec["question"],
                                    rec["ori_fake"] + rec["reranked_dense_ctxs"], [0, 1, 1, 1, 1], rec["wrong_answer"])
        ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
        out.append((enc["input_ids"][0], w[0], ans))
    return out


def test_planted_ranking_has_the_designed_boundaries():
    from transformers import AutoTokenizer
    torch.manual_seed(0)
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3"))
    spec = ModelSpec(4, 256, 8, 2, 32, 512, 8192, 1e-5, False, "llama")
    eng = CrAMEngine.random(spec, torch.device("cpu"), seed=5)
    qs = _questions(tok, (3, 5))
    lay = planted.plant_structure(eng, tiers=TIERS, bos_id=tok.bos_token_id)
    assert lay.boundaries == [3, 8, 12, 20]
    info = planted.calibrate(eng, lay, qs)
    assert (info["p_bos"] > 0.05).all() and (info["p_bos"] < 0.95).all(), info["p_bos"]

    f32 = Fp32Llama(eng)
    grids = np.stack([f32.ie_grid(ids, torch.log(w16.float()), ans).numpy() for ids, w16, ans in qs])
    mean = grids.mean(0)
    pos = np.array([mean[l, h] for l, h in lay.positive()])
    neg = np.array([mean[l, h] for l, h in lay.negative()])
    rel = np.abs(pos - lay.targets) / lay.targets
    print("\nplanted h+ IE / target:", np.round(pos / lay.targets, 4).tolist())
    assert rel.max() < 0.03, rel.max()                       # first-order calibration holds
    assert np.abs(neg + lay.targets).max() < 0.03 * lay.targets.max()
    planted_set = set(lay.positive()) | set(lay.negative())
    rest = np.array([mean[l, h] for l in range(4) for h in range(8) if (l, h) not in planted_set])
    assert np.abs(rest).max() < 0.5, np.abs(rest).max()

    ranked = Hd.rank_heads(grids)
    vals = np.array([v for v, _ in ranked])
    for k, want in planted.designed_ranking(lay, 4, 8).items():
        got = {lh for _, lh in ranked[:k]}
        assert got == want, k
        assert vals[k - 1] - vals[k] > 0.9, (k, vals[k - 1] - vals[k])
