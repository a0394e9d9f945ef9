"""Decode-attention microbench (config 2 shape): B sequences with ragged lengths, Llama-3 GQA 4:1."""
import argparse
import sys

import torch

sys.path.insert(0, '.')
from cram_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=64)
ap.add_argument("--S", type=int, default=1024)
ap.add_argument("--Hq", type=int, default=32)
ap.add_argument("--Hkv", type=int, default=8)
ap.add_argument("--splits", type=str, default="1,2,4,8")   # "," or ":" separated
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()
dev = torch.device("cuda:0")
d = 128
g = torch.Generator(device=dev).manual_seed(0)
kc = torch.randn(a.B, a.Hkv, a.S, d, device=dev, generator=g).to(torch.bfloat16)
vc = torch.randn(a.B, a.Hkv, a.S, d, device=dev, generator=g).to(torch.bfloat16)
q = torch.randn(a.B, a.Hq, d, device=dev, generator=g).to(torch.bfloat16)
lens = torch.randint(int(a.S * 0.7), a.S + 1, (a.B,), device=dev, generator=g).to(torch.int32)
kv_bytes = float(lens.sum()) * a.Hkv * d * 2 * 2
for ns in [int(x) for x in a.splits.replace(":", ",").split(",")]:
    ws = torch.empty(ops.decode_workspace_bytes(a.B, a.Hq, d, ns), dtype=torch.uint8, device=dev) if ns > 1 else None
    run = lambda: ops.attn_decode(q, kc, vc, scale=d ** -0.5, seq_lens=lens, num_splits=ns, workspace=ws)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        run()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    print(f"decode B={a.B} S<={a.S} splits={ns}: {ms * 1e3:.1f} us, {kv_bytes / (ms * 1e-3) / 1e9:.0f} GB/s (K+V bytes)")
