"""Phase timing of one batched reweighted decode (config 2 shape): host setup, packed prefill, graph capture,
graph-replayed steps, read-back.  Every phase is bracketed by torch.cuda.synchronize(), so host time and GPU
time of a phase are not separated; the rocprofv3 kernel sum of the same run gives the GPU side.

    python tools/prof_generate.py [--B 256] [--new 16] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from cram_amd import scores, spans  # noqa: E402
from cram_amd.engine import CrAMEngine, DecodeSession, ModelSpec, configure_blas  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=256)
ap.add_argument("--new", type=int, default=16)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--model", default="llama3-8b", choices=["llama3-8b", "qwen2-7b"],
                help="llama3-8b: config 2 (NQ, top-894 heads); qwen2-7b: config 4 (TriviaQA, all heads)")
a = ap.parse_args()

dev = torch.device("cuda:0")
configure_blas("hipblaslt")
qwen = a.model == "qwen2-7b"
spec = ModelSpec.qwen2_7b() if qwen else ModelSpec.llama3_8b()
eng = CrAMEngine.random(spec, dev, seed=1234, rope_theta=1e6 if qwen else 500000.0)
from transformers import AutoTokenizer  # noqa: E402
import gzip  # noqa: E402
tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_qwen" if qwen else "tok_llama3"))
data = json.load(gzip.open(os.path.join(REPO, "data", ("trivia" if qwen else "nq") + "_1000.json.gz"), "rt",
                           encoding="utf-8"))
heads = {} if qwen else json.load(open(os.path.join(REPO, "data", "selected_heads.json")))["nq__llama3"]["heads"]
qs, ps, ss = [], [], []
for j in range(a.B):
    paras, sc = scores.assemble(data[j], ideal=True, ideal_score=1)
    qs.append(data[j]["question"]); ps.append(paras); ss.append(sc)
encs = spans.encode_batch(tok, "Qwen2-7B-Instruct" if qwen else "Meta-Llama-3-8B-Instruct", qs, ps, ss)
prompts = [ids.to(dev) for ids, _, _ in encs]
ws = [w for _, w, _ in encs]


def sync_t():
    torch.cuda.synchronize()
    return time.perf_counter()


for rep in range(a.reps):
    t = [sync_t()]
    sess = DecodeSession(eng, prompts, ws, heads, a.new)
    t.append(sync_t())
    sess.prefill()
    t.append(sync_t())
    sess.capture()
    t.append(sync_t())
    for _ in range(a.new - 1):
        sess.step(True)
    t.append(sync_t())
    out = sess.generated().cpu().tolist()
    t.append(sync_t())
    names = ["session", "prefill", "capture", "steps", "readback"]
    ph = {n: round((t[i + 1] - t[i]) * 1e3, 1) for i, n in enumerate(names)}
    print(f"rep {rep}: total {(t[-1] - t[0]) * 1e3:.0f} ms  " + "  ".join(f"{k} {v}" for k, v in ph.items()), flush=True)
    del sess
