"""Top-k head-set identity at the k the path uses, Llama-3-8B shape, full 32 x 32 grids.

For NQ questions (random-init Llama-3-8B weights: no checkpoint offline; sweep scores [0, 1, 1, 1, 1],
find_best_heads.py:41-50) three IE grids [Nq, 32, 32] are computed on one MI355X:
  ours   the head-batched layer-suffix sweep (cram_amd.sweep.ie_question, the path bench.py times)
  ref    the reference algorithm itself in bf16: transformers LlamaForCausalLM + the dense-mask pre-hook
         (oracle/hook_ref.py, bit-exact to re_weighting.py on CPU), one hooked forward + fp32-upcast answer
         logits per unit (re_weighting.py:152-175)
  truth  float32 PyTorch with the hook's dense mask (tests/fp32_llama.py, per-layer batched)
Each grid is ranked the way find_best_heads.py:113-150 ranks (mean over questions, descending, fixed tie-break
cram_amd.heads.rank_heads) and the top-k sets are compared at k = 894 (nq/llama3), 506 (trivia/llama3), 100, 10.
For every k: set overlaps ours/truth, ref/truth, ours/ref; the truth's boundary gap (k-th minus (k+1)-th mean
IE); the bf16 noise of the mean (max |mean_ours - mean_truth|, same for ref); identity is guaranteed for a
bf16 run whenever gap > 2 x its noise.
Usage (GPU box):  python tools/topk_identity.py [n_questions] > profiles/r02_topk_identity.json
"""
from __future__ import annotations

import gzip
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from cram_amd import heads as Hd  # noqa: E402
from cram_amd import spans, sweep  # noqa: E402
from cram_amd.engine import CrAMEngine, ModelSpec  # noqa: E402

KS = (894, 506, 100, 10)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def topk_set(grid, k):
    return {lh for _, lh in Hd.rank_heads(grid)[:k]}


def compare(ours, ref, truth):
    mt, mo, mr = truth.mean(0).reshape(-1), ours.mean(0).reshape(-1), ref.mean(0).reshape(-1)
    st = np.sort(mt)[::-1]
    noise_o, noise_r = float(np.abs(mo - mt).max()), float(np.abs(mr - mt).max())
    rows = {}
    for k in KS:
        T, O, R = topk_set(truth, k), topk_set(ours, k), topk_set(ref, k)
        gap = float(st[k - 1] - st[k])
        rows[k] = {"ours_vs_truth": len(O & T), "ref_vs_truth": len(R & T), "ours_vs_ref": len(O & R),
                   "truth_boundary_gap": gap, "identity_guaranteed_ours": gap > 2 * noise_o,
                   "identity_guaranteed_ref": gap > 2 * noise_r, "ours_identical_to_truth": O == T,
                   "ref_identical_to_truth": R == T}
    return {"mean_abs_ie_truth": float(np.abs(mt).mean()), "noise_ours_max": noise_o, "noise_ref_max": noise_r,
            "noise_ours_mean": float(np.abs(mo - mt).mean()), "noise_ref_mean": float(np.abs(mr - mt).mean()),
            "topk": rows}


def main():
    nq_n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    from transformers import AutoTokenizer
    from oracle import cpu_baseline, hook_ref
    from tests.fp32_llama import Fp32Llama
    dev = torch.device("cuda:0")
    eng = CrAMEngine.random(ModelSpec.llama3_8b(), dev, seed=1234, rope_theta=500000.0)
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3"))
    data = json.load(gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8"))
    qs = list(range(3, 3 + nq_n))
    ours, ref, truth, meta = [], [], [], []
    hf = cpu_baseline.hf_model_from_engine(eng).to(dev)
    f32 = Fp32Llama(eng)
    for qi in qs:
        rec = data[qi]
        _, enc, w, _ = spans.encode(tok, "Meta-Llama-3-8B-Instruct", rec["question"],
                                    rec["ori_fake"] + rec["reranked_dense_ctxs"], [0, 1, 1, 1, 1], rec["wrong_answer"])
        ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:].to(dev)
        ids, w16 = enc["input_ids"][0].to(dev), w[0]
        t0 = time.time()
        ours.append(sweep.ie_question(eng, ids, w16, ans).double().cpu().numpy())
        torch.cuda.synchronize()
        t1 = time.time()
        log(f"question {qi}: sweep done ({t1 - t0:.1f}s)")
        lw = hook_ref.log_weight(w16.view(1, -1)).to(dev)
        ref.append(hook_ref.ie_grid(hf, ids[None], lw, ans, upcast_logits=True))
        torch.cuda.synchronize()
        t2 = time.time()
        log(f"question {qi}: reference hook grid done ({t2 - t1:.1f}s)")
        truth.append(f32.ie_grid(ids, torch.log(w16.to(dev).float()), ans).numpy())
        torch.cuda.synchronize()
        t3 = time.time()
        meta.append({"question": qi, "T": int(ids.numel()), "n_ans": int(ans.numel()),
                     "seconds": {"ours": round(t1 - t0, 2), "ref": round(t2 - t1, 2), "truth": round(t3 - t2, 2)}})
        log(f"question {qi}: T'={ids.numel()} ours {t1 - t0:.1f}s ref {t2 - t1:.1f}s truth {t3 - t2:.1f}s; "
            f"per-question |ours-truth| mean {np.abs(ours[-1] - truth[-1]).mean():.4f}, "
            f"|ref-truth| mean {np.abs(ref[-1] - truth[-1]).mean():.4f}")
    O, R, T = np.stack(ours), np.stack(ref), np.stack(truth)
    res = {"shape": "Llama-3-8B (random init, seed 1234), NQ questions " + ",".join(map(str, qs)),
           "questions": meta, "all": compare(O, R, T),
           "per_question_noise": [{"ours_mean": float(np.abs(O[i] - T[i]).mean()),
                                   "ref_mean": float(np.abs(R[i] - T[i]).mean())} for i in range(len(qs))]}
    np.savez_compressed(os.path.join(REPO, "gpurun_out", "topk_identity_grids.npz"), ours=O, ref=R, truth=T)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
