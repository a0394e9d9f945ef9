"""Does row-chunking the MLP (gate/up GEMM -> SiLU-mul -> down GEMM) keep the [rows, 2F] intermediate in the
256 MB Infinity Cache and pay for the smaller GEMMs?  Same-process interleaved A/B at M = 28672 (Llama-3-8B).

    python tools/mlp_chunk_probe.py
"""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cram_amd import build, gemm_tune, ops  # noqa: E402

if build.needs_build():
    build.build()
gemm_tune.ensure()
dev = torch.device("cuda:0")
M, D, Fi = 28672, 4096, 14336
x = torch.randn(M, D, device=dev).to(torch.bfloat16)
wgu = (torch.randn(2 * Fi, D, device=dev) * 0.02).to(torch.bfloat16)
wd = (torch.randn(D, Fi, device=dev) * 0.02).to(torch.bfloat16)
out = torch.empty(M, D, device=dev, dtype=torch.bfloat16)


def mlp(chunk):
    for r0 in range(0, M, chunk):
        xs = x[r0:r0 + chunk]
        act = ops.silu_mul(F.linear(xs, wgu), Fi)
        torch.matmul(act, wd.t(), out=out[r0:r0 + chunk])


variants = [M, 14336, 8192, 4096]
res = {c: [] for c in variants}
for rnd in range(6):
    for c in variants:
        mlp(c)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(4):
            mlp(c)
        e.record()
        torch.cuda.synchronize()
        res[c].append(s.elapsed_time(e) / 4)
for c in variants:
    print(f"MLP M={M} in chunks of {c}: {statistics.median(res[c]):.3f} ms", flush=True)
