"""Standalone driver of the IE-sweep attention shape for rocprofv3 (kernel trace / PMC passes)."""
import argparse
import sys

import torch

sys.path.insert(0, '.')
from cram_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=33)
ap.add_argument("--T", type=int, default=962)
ap.add_argument("--Hq", type=int, default=32)
ap.add_argument("--Hkv", type=int, default=8)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--biased", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
d = 128
N = (a.Hq + 2 * a.Hkv) * d
y = torch.randn(a.B, a.T, N, device=dev).to(torch.bfloat16)       # fused QKV buffer, token-major
q = y[..., :a.Hq * d].unflatten(-1, (a.Hq, d)).transpose(1, 2)
k = y[..., a.Hq * d:(a.Hq + a.Hkv) * d].unflatten(-1, (a.Hkv, d)).transpose(1, 2)
v = y[..., (a.Hq + a.Hkv) * d:].unflatten(-1, (a.Hkv, d)).transpose(1, 2)
bias = enable = None
if a.biased:
    bias = torch.zeros(a.B, a.T, device=dev)
    bias[:, 40:200] = float("-inf")
    enable = torch.ones(a.B, a.Hq, dtype=torch.uint8, device=dev)
out = torch.empty(a.B, a.T, a.Hq, d, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    ops.attn_prefill(q, k, v, scale=d ** -0.5, bias=bias, enable=enable, W=a.T if a.biased else 0, out=out)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(a.iters):
    ops.attn_prefill(q, k, v, scale=d ** -0.5, bias=bias, enable=enable, W=a.T if a.biased else 0, out=out)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / a.iters
fl, by = ops.prefill_work(a.B, a.Hq, a.Hkv, a.T, a.T, d, 0)
print(f"attn B={a.B} T={a.T} Hq={a.Hq} Hkv={a.Hkv}: {ms:.3f} ms/launch, {fl / ms / 1e9:.1f} TFLOP/s, "
      f"{by / ms / 1e6:.1f} GB/s algorithmic")
