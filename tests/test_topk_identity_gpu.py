"""Top-k head-set identity at the Llama-3-8B shape, asserted (north star: "the resulting top-k head ranking is
bit-identical").

The model is random-init Llama-3-8B with a planted set of 130 head pairs whose IE (re_weighting.py:152-175) is large,
sign-controlled and tiered (tests/planted.py; the construction is checked against the float32 truth on a tiny model
in tests/test_planted_cpu.py).  For 4 rebuilt NQ questions (sweep scores [0, 1, 1, 1, 1], find_best_heads.py:41-50)
three full 32 x 32 IE grids are computed on the GPU:
  ours   the head-batched layer-suffix sweep (cram_amd.sweep.ie_question, the path bench.py times)
  ref    the reference algorithm itself in bf16: transformers LlamaForCausalLM + the dense-mask pre-hook
         (oracle/hook_ref.py, bit-exact to re_weighting.py on CPU), one hooked forward + fp32-upcast answer logits
         per unit
  truth  float32 PyTorch with the hook's dense mask (tests/fp32_llama.py)
Each is ranked as find_best_heads.py:113-150 ranks (mean over questions, descending; cram_amd.heads.rank_heads).
Bar: at EVERY k in 1..1023 where the truth's boundary gap (k-th minus (k+1)-th mean IE) exceeds 3x the larger of the
two bf16 runs' max |mean IE - truth|, top-k(ours) == top-k(ref) == top-k(truth).  The test fails unless at least 3
such k exist, one of them >= 100, and the path's own k = 894 (datasets/nq/llama3/selected_heads.json) is among them.
The random-weight noise-floor tests stay in tests/test_fullsize_ie_gpu.py.
"""
import gzip
import json
import os
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUESTIONS = (3, 4, 5, 6)
PATH_K = 894
_GRIDS = {}


@pytest.fixture(scope="module")
def planted_model(gpu_device):
    from transformers import AutoTokenizer

    from cram_amd import spans
    from cram_amd.engine import CrAMEngine, ModelSpec
    from oracle import cpu_baseline
    from tests import planted
    from tests.fp32_llama import Fp32Llama

    dev = gpu_device
    eng = CrAMEngine.random(ModelSpec.llama3_8b(), dev, seed=1234, rope_theta=500000.0)
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3"))
    data = json.load(gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8"))
    qs = []
    for i in QUESTIONS:
        rec = data[i]
        _, enc, w, _ = spans.encode(tok, "Meta-Llama-3-8B-Instruct", rec["question"],
                                    rec["ori_fake"] + rec["reranked_dense_ctxs"], [0, 1, 1, 1, 1], rec["wrong_answer"])
        ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
        qs.append((enc["input_ids"][0].to(dev), w[0].to(dev), ans.to(dev)))
    lay = planted.plant_structure(eng, bos_id=tok.bos_token_id)
    info = planted.calibrate(eng, lay, qs)
    print(f"\nplanted {len(lay.pairs)} pairs; mean p_BOS {info['p_bos'].mean():.3f} "
          f"(min {info['p_bos'].min():.3f}, max {info['p_bos'].max():.3f}); designed boundaries {lay.boundaries}")
    hf = cpu_baseline.hf_model_from_engine(eng).to(dev)
    f32 = Fp32Llama(eng)
    yield eng, qs, lay, hf, f32
    del hf, f32, eng
    _GRIDS.clear()
    torch.cuda.empty_cache()


def _grids(planted_model, i):
    if i not in _GRIDS:
        from cram_amd import sweep
        from oracle import hook_ref
        eng, qs, _, hf, f32 = planted_model
        ids, w16, ans = qs[i]
        t0 = time.time()
        ours = sweep.ie_question(eng, ids, w16, ans).double().cpu().numpy()
        t1 = time.time()
        ref = hook_ref.ie_grid(hf, ids[None], hook_ref.log_weight(w16.view(1, -1)), ans, upcast_logits=True)
        t2 = time.time()
        truth = f32.ie_grid(ids, torch.log(w16.float()), ans).numpy()
        t3 = time.time()
        print(f"\nquestion {QUESTIONS[i]}: T'={ids.numel()} n={ans.numel()}  ours {t1 - t0:.1f}s ref {t2 - t1:.1f}s "
              f"truth {t3 - t2:.1f}s; |ours-truth| max {np.abs(ours - truth).max():.4f} "
              f"|ref-truth| max {np.abs(ref - truth).max():.4f}")
        _GRIDS[i] = (ours, ref, truth)
    return _GRIDS[i]


@pytest.mark.parametrize("i", range(len(QUESTIONS)))
def test_planted_question_grids(planted_model, i):
    """One question's three grids (kept for the identity test; split so each test reports within ~90 s)."""
    ours, ref, truth = _grids(planted_model, i)
    assert np.isfinite(ours).all() and np.isfinite(ref).all() and np.isfinite(truth).all()
    _, _, lay, _, _ = planted_model
    pos = np.array([truth[l, h] for l, h in lay.positive()])
    assert (pos > 0).all(), "every planted h+ has a positive IE in the float32 truth"


def test_planted_topk_identity_at_every_separated_k(planted_model):
    from cram_amd import heads as Hd
    _, _, lay, _, _ = planted_model
    G = [_grids(planted_model, i) for i in range(len(QUESTIONS))]
    O, R, T = (np.stack([g[j] for g in G]) for j in range(3))
    mo, mr, mt = O.mean(0).reshape(-1), R.mean(0).reshape(-1), T.mean(0).reshape(-1)
    noise_o, noise_r = float(np.abs(mo - mt).max()), float(np.abs(mr - mt).max())
    bar = 3.0 * max(noise_o, noise_r)
    ro, rr, rt = Hd.rank_heads(O), Hd.rank_heads(R), Hd.rank_heads(T)
    vt = np.array([v for v, _ in rt])
    asserted, failed = [], []
    for k in range(1, vt.size):
        if vt[k - 1] - vt[k] > bar:
            so, sr, st = ({lh for _, lh in r[:k]} for r in (ro, rr, rt))
            asserted.append(k)
            if not (so == st and sr == st):
                failed.append((k, len(so & st), len(sr & st)))
    pos = np.array([T.mean(0)[l, h] for l, h in lay.positive()])
    summary = {"questions": list(QUESTIONS), "noise_ours_max": noise_o, "noise_ref_max": noise_r, "bar": bar,
               "noise_ours_mean": float(np.abs(mo - mt).mean()), "noise_ref_mean": float(np.abs(mr - mt).mean()),
               "planted_ie_over_target": [float(x) for x in np.round(pos / lay.targets, 4)],
               "designed_boundaries": lay.boundaries, "asserted_k": asserted, "failed": failed,
               "gap_at_designed": {k: float(vt[k - 1] - vt[k]) for k in lay.boundaries},
               "margin_at_designed": {k: float(vt[k - 1] - vt[k]) / bar for k in lay.boundaries},
               "random_heads_max_abs_ie": float(np.abs(np.delete(mt, [l * T.shape[2] + h for l, h in
                                                                      lay.positive() + lay.negative()])).max())}
    print("\n" + json.dumps(summary))
    if os.environ.get("CRAM_TOPK_OUT"):
        with open(os.environ["CRAM_TOPK_OUT"], "w") as f:
            json.dump(summary, f, indent=1)
        np.savez_compressed(os.environ["CRAM_TOPK_OUT"] + ".npz", ours=O, ref=R, truth=T)
    margins = {k: float(vt[k - 1] - vt[k]) / bar for k in lay.boundaries}
    print("margin (truth gap / bar) at the designed boundaries: " + json.dumps({k: round(v, 3) for k, v in margins.items()}))
    assert not failed, failed
    assert len(asserted) >= 3 and max(asserted) >= 100, asserted
    assert PATH_K in asserted, (PATH_K, asserted)
    # every designed boundary (tier edges 10 / 50 / 100, the 130 planted h+, the path's 894) is asserted, with the
    # truth's gap at least 1.5 x the 3 x noise bar
    assert set(lay.boundaries) <= set(asserted), (lay.boundaries, asserted)
    assert min(margins.values()) >= 1.5, margins
