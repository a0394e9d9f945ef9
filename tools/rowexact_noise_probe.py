"""IE error against the float32 truth with and without the row-exact baseline (sweep.ROW_EXACT), over several NQ
questions at the Llama-3-8B shape (random-init weights, as tests/test_fullsize_ie_gpu.py): per question the sweep in
both modes, the reference algorithm in bf16 (transformers + the dense-mask hook, oracle/hook_ref.py) and the float32
truth (tests/fp32_llama.py) on layers 0 / 13 / 31 x 32 heads.  Prints mean / max / RMS |IE - truth| per question and
the totals.  Diagnostics only.

  python tools/rowexact_noise_probe.py [first question] [count]
"""
import gzip
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from transformers import AutoTokenizer  # noqa: E402

from cram_amd import spans, sweep  # noqa: E402
from cram_amd.engine import CrAMEngine, ModelSpec  # noqa: E402
from oracle import cpu_baseline, hook_ref  # noqa: E402
from tests.fp32_llama import Fp32Llama  # noqa: E402

LAYERS = (0, 13, 31)


def topk_overlap(g, truth, k):
    from cram_amd import heads as Hd
    top = lambda x: {lh for _, lh in Hd.rank_heads(x.reshape(1, 32, 32).numpy())[:k]}
    return len(top(g) & top(truth))


def main():
    q0 = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    nq = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    grid = len(sys.argv) > 3 and sys.argv[3] == "grid"      # all 32 layers: the top-k overlaps of the grid test
    global LAYERS
    if grid:
        LAYERS = tuple(range(32))
    dev = torch.device("cuda:0")
    eng = CrAMEngine.random(ModelSpec.llama3_8b(), dev, seed=1234, rope_theta=500000.0)
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3"))
    data = json.load(gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8"))
    H = eng.spec.num_heads
    units = [(l, h) for l in LAYERS for h in range(H)]
    hook_layers = None if grid else LAYERS
    tot = {k: [] for k in ("re1", "re0", "hook")}
    for qi in range(q0, q0 + nq):
        rec = data[qi]
        _, enc, w, _ = spans.encode(tok, "Meta-Llama-3-8B-Instruct", rec["question"],
                                    rec["ori_fake"] + rec["reranked_dense_ctxs"], [0, 1, 1, 1, 1], rec["wrong_answer"])
        ids, w16 = enc["input_ids"][0].to(dev), w[0]
        ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:].to(dev)
        out = {}
        for mode in ("re1", "re0"):
            sweep.ROW_EXACT = mode == "re1"
            out[mode] = sweep.ie_question(eng, ids, w16, ans, layers=None if grid else LAYERS).double().cpu().flatten()
        sweep.ROW_EXACT = True
        hf = cpu_baseline.hf_model_from_engine(eng).to(dev)
        out["hook"] = torch.tensor(hook_ref.ie_grid(hf, ids[None], hook_ref.log_weight(w16.view(1, -1)).to(dev), ans,
                                                    layers=hook_layers, upcast_logits=True), dtype=torch.float64).flatten()
        del hf
        f32 = Fp32Llama(eng)
        if grid:
            truth = f32.ie_grid(ids, torch.log(w16.to(dev).float()), ans).double().flatten()
        else:
            truth = torch.tensor(f32.ie_units(ids, torch.log(w16.to(dev).float()), ans, units), dtype=torch.float64)
        del f32
        torch.cuda.empty_cache()
        line = [f"q{qi} T'={ids.numel()} |IE| mean {truth.abs().mean():.4f}"]
        for k in ("re1", "re0", "hook"):
            e = (out[k] - truth).abs()
            tot[k].append(e)
            line.append(f"{k}: mean {e.mean():.4f} max {e.max():.4f} rms {e.pow(2).mean().sqrt():.4f}")
        line.append(f"|re1-re0| max {(out['re1'] - out['re0']).abs().max():.4f}")
        if grid:
            for k in (894, 506, 100, 10):
                line.append(f"k={k} " + " ".join(f"{m} {topk_overlap(out[m], truth, k)}" for m in ("re1", "re0", "hook")))
        print(" | ".join(line), flush=True)
    print("all questions:")
    for k, es in tot.items():
        e = torch.cat(es)
        print(f"  {k}: mean {e.mean():.5f} max {e.max():.4f} rms {e.pow(2).mean().sqrt():.5f}")


if __name__ == "__main__":
    main()
