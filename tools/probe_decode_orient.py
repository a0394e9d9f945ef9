"""Decode-step GEMM orientation probe: F.linear(x [M, K], w [N, K]) (the step's form, M = batch rows) against the
transposed product w @ x^T ([N, M], then one transpose copy back), cold caches (weight copies cycled past the
256 MB MALL), default heuristic, same process, medians.   python tools/probe_decode_orient.py [M]"""
import statistics
import sys

import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
shapes = [("qkv", 4096, 6144), ("o", 4096, 4096), ("gate/up", 4096, 28672), ("down", 14336, 4096),
          ("qwen o", 3584, 3584), ("qwen gate/up", 3584, 37888), ("qwen down", 18944, 3584)]


def bench(fn, ws, x):
    for w in ws:
        fn(x, w)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(20):
        fn(x, ws[i % len(ws)])
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 20 * 1e3


lin = lambda x, w: F.linear(x, w)
tr = lambda x, w: torch.mm(w, x.t()).t().contiguous()
tr_nc = lambda x, w: torch.mm(w, x.t())
for name, K, N in shapes:
    nc = min(16, max(2, -(-768 * 2**20 // (N * K * 2))))
    ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(nc)]
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    ref = F.linear(x, ws[0]).float()
    assert (tr(x, ws[0]).float() - ref).abs().max().item() < 0.1
    r = {k: [] for k in ("linear", "w@x^T+copy", "w@x^T")}
    for _ in range(5):
        r["linear"].append(bench(lin, ws, x))
        r["w@x^T+copy"].append(bench(tr, ws, x))
        r["w@x^T"].append(bench(tr_nc, ws, x))
    gb = N * K * 2 / 1e9
    print(f"{name:13s} M={M} K={K:5d} N={N:6d} " + "  ".join(
        f"{k} {statistics.median(v):6.1f} us ({gb / statistics.median(v) * 1e6 / 1e3:4.2f} TB/s)" for k, v in r.items()),
        flush=True)
