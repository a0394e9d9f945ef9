"""Numerics of the pinned decode-step GEMM solutions (data/gemm_solutions.json decode_solutions) against the default
pick: max / mean |C - C_fp32| over random bf16 operands of each pinned (N, K, M), where C_fp32 is the float32 product
of the same bf16 operands.  TunableOp does not check numerics when it tunes; a split-K pick with 16-bit partials would
show here.   python tools/check_decode_pins.py"""
import json
import os

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import sys  # noqa: E402
sys.path.insert(0, REPO)
from cram_amd import gemm_tune  # noqa: E402

dev = torch.device("cuda:0")
sol = gemm_tune.load()
assert gemm_tune.ensure(), "pins not installed (other build?)"
tun = torch.cuda.tunable
for key, name in sol.get("decode_solutions", {}).items():
    N, K, M = (int(v) for v in key.split("x"))
    g = torch.Generator(device=dev).manual_seed(N + K + M)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    d = F.linear(x, w).float()
    with gemm_tune.pinned(decode=True):
        pnd = F.linear(x, w).float()
    ed, ep = (d - ref).abs(), (pnd - ref).abs()
    print(f"{key:18s} {name:24s} default max {ed.max():.3e} mean {ed.mean():.3e} | pinned max {ep.max():.3e} "
          f"mean {ep.mean():.3e} | ratio mean {ep.mean() / ed.mean():.3f}", flush=True)
