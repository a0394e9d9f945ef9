"""Accuracy of the IE sweep's baseline cache in its two forms (sweep.baseline with and without the row-exact mode)
against the float32 forward (tests/fp32_llama.py) on one NQ question at the Llama-3-8B shape: per layer the relative
RMS error of the cached layer input h_l, and of the final hidden states of the answer rows.  Diagnostics only.

  python tools/baseline_cache_probe.py [question]
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
from cram_amd.bias import CredibilityBias  # noqa: E402
from cram_amd.engine import CrAMEngine, ModelSpec  # noqa: E402
from tests.fp32_llama import Fp32Llama  # noqa: E402


def main():
    qi = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    eng = CrAMEngine.random(ModelSpec.llama3_8b(), dev, seed=1234, rope_theta=500000.0)
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3"))
    data = json.load(gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8"))
    rec = data[qi]
    _, enc, w, _ = spans.encode(tok, "Meta-Llama-3-8B-Instruct", rec["question"],
                                rec["ori_fake"] + rec["reranked_dense_ctxs"], [0, 1, 1, 1, 1], rec["wrong_answer"])
    ids, w16 = enc["input_ids"][0].to(dev), w[0]
    n = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:].numel()
    sp = eng.spec
    cb = CredibilityBias.build([w16.view(1, -1)], {}, sp.num_layers, sp.num_heads, dev, eng.dtype)
    p0 = sweep.first_biased_row(cb.bias, cb.W)
    caches = {}
    for mode in ("re1", "re0"):
        sweep.ROW_EXACT = mode == "re1"
        caches[mode] = sweep.baseline(eng, ids, n, p0=p0)
    sweep.ROW_EXACT = True
    hs32, hf32 = Fp32Llama(eng).baseline(ids)
    rel = lambda a, b: float((a.float() - b).pow(2).mean().sqrt() / b.pow(2).mean().sqrt())
    print(f"q{qi} T'={ids.numel()} p0={p0} n={n}")
    for l in range(0, sp.num_layers, 4):
        print(f"  h_in[{l:2d}] rel rms err: re1 {rel(caches['re1'][1].h_in[l][0], hs32[l]):.3e}  "
              f"re0 {rel(caches['re0'][1].h_in[l][0], hs32[l]):.3e}  "
              f"re1 vs re0 {rel(caches['re1'][1].h_in[l][0], caches['re0'][1].h_in[l][0].float()):.3e}")
    print(f"  final answer rows rel rms err: re1 {rel(caches['re1'][0], hf32[-n:]):.3e}  "
          f"re0 {rel(caches['re0'][0], hf32[-n:]):.3e}")
    for l in (0, 13, 31):
        a1, a0 = caches["re1"][1].a[l][0, -n:].float(), caches["re0"][1].a[l][0, -n:].float()
        print(f"  attention out layer {l} (answer rows) re1 vs re0 rel {rel(a1, a0):.3e}")


if __name__ == "__main__":
    main()
