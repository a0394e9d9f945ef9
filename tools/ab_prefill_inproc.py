"""Same-process interleaved A/B of prefill-kernel variants (the library's CRAM_KNOB_PREFILL_VARIANT knob, -1 / 3 / 8):
N rounds x variants x shapes, median ms per launch.  Usage: python tools/ab_prefill_inproc.py -1 3 8"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cram_amd import _lib, ops  # noqa: E402

variants = sys.argv[1:] or ["-1", "8"]
dev = torch.device("cuda:0")
d = 128
# AB_HEADS=28,4 for the Qwen2-7B head layout (GQA 7)
HQ, HKV = (int(x) for x in os.environ.get("AB_HEADS", "32,8").split(","))
shapes = [(33, 962), (1, 8300)]
data = {}
for B, T in shapes:
    y = torch.randn(B, T, (HQ + 2 * HKV) * d, device=dev).to(torch.bfloat16)
    q = y[..., :HQ * d].unflatten(-1, (HQ, d)).transpose(1, 2)
    k = y[..., HQ * d:(HQ + HKV) * d].unflatten(-1, (HKV, d)).transpose(1, 2)
    v = y[..., (HQ + HKV) * d:].unflatten(-1, (HKV, d)).transpose(1, 2)
    data[(B, T)] = (q, k, v, torch.empty(B, T, HQ, d, device=dev, dtype=torch.bfloat16))
res = {(vv, s): [] for vv in variants for s in shapes}
for rnd in range(5):
    for vv in variants:
        _lib.set_knob(_lib.KNOB_PREFILL_VARIANT, int(vv))
        for s in shapes:
            q, k, v, out = data[s]
            for _ in range(2):
                ops.attn_prefill(q, k, v, scale=d ** -0.5, out=out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.attn_prefill(q, k, v, scale=d ** -0.5, out=out)
            e1.record()
            torch.cuda.synchronize()
            res[(vv, s)].append(e0.elapsed_time(e1) / 10)
for vv in variants:
    line = []
    for B, T in shapes:
        ms = statistics.median(res[(vv, (B, T))])
        fl, _ = ops.prefill_work(B, HQ, HKV, T, T, d, 0)
        line.append(f"B={B} T={T}: {ms:.3f} ms {fl / ms / 1e9:.0f} TF")
    print(f"variant {vv:>3}: " + " | ".join(line), flush=True)
