"""Full 32 x 32 IE grids at the Llama-3-8B shape for the multi-question top-k bar (tests/test_fullsize_ie_gpu.py).

Test tooling (imports the oracle as the checker).  For NQ questions q0 .. q0 + n - 1 on the bench's random-init
Llama-3-8B (CrAMEngine.random seed 1234, the fixture the GPU tests build), computes
  truth  the float32 PyTorch IE grid (tests/fp32_llama.py, dense hook mask, per-layer batched variants)
  hook   the reference algorithm itself in bf16: transformers LlamaForCausalLM + the dense-mask pre-hook
         (oracle/hook_ref.py, re_weighting.py:152-175), fp32-upcast logits
and writes one npz per question (truth, hook, T', answer ids, a checksum of the engine's weights) into OUT; the
sweep's own grids in both modes (default, row-exact) are printed beside them.  The npz files are merged into
tests/golden/fullsize_grids_llama3_8b.npz by `python tools/fullsize_grids.py merge OUT`.

  python tools/fullsize_grids.py Q0 N OUT
"""
import gzip
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def weights_checksum(eng) -> np.ndarray:
    """A strided sample of every layer's weights and of the embedding / lm_head, summed in float64 on the host:
    equal iff the random-init engine is the one the grids were computed on (deterministic torch RNG on the GPU)."""
    parts = []
    for lw in eng.layers:
        for t in (lw.wqkv, lw.wo, lw.wgu, lw.wd):
            parts.append(float(t[::97, ::89].double().sum()))
    parts.append(float(eng.embed[::997, ::13].double().sum()))
    parts.append(float(eng.lm_head[::997, ::13].double().sum()))
    return np.array(parts, dtype=np.float64)


def question(tok, data, qi, dev):
    from cram_amd import spans
    rec = data[qi]
    _, enc, w, _ = spans.encode(tok, "Meta-Llama-3-8B-Instruct", rec["question"],
                                rec["ori_fake"] + rec["reranked_dense_ctxs"], [0, 1, 1, 1, 1], rec["wrong_answer"])
    ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
    return enc["input_ids"][0].to(dev), w[0], ans.to(dev)


def main():
    if sys.argv[1] == "merge":
        src = sys.argv[2]
        fs = sorted(f for f in os.listdir(src) if f.startswith("grid_q") and f.endswith(".npz"))
        ds = [dict(np.load(os.path.join(src, f))) for f in fs]
        ds.sort(key=lambda d: int(d["qi"]))
        ck = ds[0]["checksum"]
        assert all(np.array_equal(d["checksum"], ck) for d in ds), "grids from different engines"
        out = os.path.join(REPO, "tests", "golden", "fullsize_grids_llama3_8b.npz")
        np.savez_compressed(out, qi=np.array([int(d["qi"]) for d in ds]), T=np.array([int(d["T"]) for d in ds]),
                            truth=np.stack([d["truth"] for d in ds]).astype(np.float32),
                            hook=np.stack([d["hook"] for d in ds]).astype(np.float32), checksum=ck)
        print("merged", [int(d["qi"]) for d in ds], "->", out)
        return
    q0, n, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    os.makedirs(out, exist_ok=True)
    from transformers import AutoTokenizer
    from cram_amd import sweep
    from cram_amd.engine import CrAMEngine, ModelSpec
    from oracle import cpu_baseline, hook_ref
    from tests.fp32_llama import Fp32Llama
    dev = torch.device("cuda:0")
    eng = CrAMEngine.random(ModelSpec.llama3_8b(), dev, seed=1234, rope_theta=500000.0)
    ck = weights_checksum(eng)
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3"))
    data = json.load(gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8"))
    for qi in range(q0, q0 + n):
        t0 = time.time()
        ids, w16, ans = question(tok, data, qi, dev)
        hf = cpu_baseline.hf_model_from_engine(eng).to(dev)
        hook = hook_ref.ie_grid(hf, ids[None], hook_ref.log_weight(w16.view(1, -1)).to(dev), ans, upcast_logits=True)
        del hf
        torch.cuda.empty_cache()
        t1 = time.time()
        f32 = Fp32Llama(eng)
        truth = f32.ie_grid(ids, torch.log(w16.to(dev).float()), ans).numpy()
        del f32
        torch.cuda.empty_cache()
        t2 = time.time()
        mine = {}
        for mode in (False, True):
            sweep.ROW_EXACT = mode
            mine[mode] = sweep.ie_question(eng, ids, w16, ans).double().cpu().numpy()
        sweep.ROW_EXACT = False
        np.savez(os.path.join(out, f"grid_q{qi}.npz"), qi=qi, T=ids.numel(), truth=truth, hook=np.asarray(hook),
                 ans=ans.cpu().numpy(), checksum=ck)
        rms = lambda g: float(np.sqrt(((g - truth) ** 2).mean()))
        print(f"q{qi} T'={ids.numel()} hook {t1 - t0:.0f}s truth {t2 - t1:.0f}s | rms hook {rms(hook):.4f} "
              f"default {rms(mine[False]):.4f} row-exact {rms(mine[True]):.4f}", flush=True)


if __name__ == "__main__":
    main()
