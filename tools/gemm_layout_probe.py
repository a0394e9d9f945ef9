"""Weight layout of the sweep's projection GEMMs: F.linear's [N, K] weights (hipBLASLt 'TN', both operands
K-contiguous) against the same weights stored [K, N] (x @ Wt, 'NN'), at the IE sweep's row count, same process,
interleaved rounds, medians; weights cycled over 4 copies so each call reads them from HBM as the sweep does.
Also checks the two layouts give identical results (the same dot products; only the kernel differs).
  python tools/gemm_layout_probe.py [M]"""
import statistics
import sys

import torch

M = int(sys.argv[1]) if len(sys.argv) > 1 else 29184
dev = torch.device("cuda:0")
torch.backends.cuda.preferred_blas_library("hipblaslt")
shapes = {"qkv": (6144, 4096), "o_proj": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
g = torch.Generator(device=dev).manual_seed(0)
res = {}
for name, (N, K) in shapes.items():
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    ws = [(torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16) for _ in range(4)]
    wts = [w.t().contiguous() for w in ws]
    a = torch.nn.functional.linear(x, ws[0])
    b = x @ wts[0]
    same = bool(torch.equal(a, b))
    dmax = (a.float() - b.float()).abs().max().item()
    t = {"TN": [], "NN": []}
    for _ in range(7):
        for lay in ("TN", "NN"):
            for i in range(4):
                (torch.nn.functional.linear(x, ws[i]) if lay == "TN" else x @ wts[i])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for r in range(8):
                i = r % 4
                (torch.nn.functional.linear(x, ws[i]) if lay == "TN" else x @ wts[i])
            e1.record()
            torch.cuda.synchronize()
            t[lay].append(e0.elapsed_time(e1) / 8)
    fl = 2.0 * M * N * K
    tn, nn = statistics.median(t["TN"]), statistics.median(t["NN"])
    print(f"{name:8s} M={M} N={N} K={K}: TN {tn:.3f} ms ({fl / tn / 1e9:.0f} TF/s)  NN {nn:.3f} ms "
          f"({fl / nn / 1e9:.0f} TF/s)  NN/TN speed {tn / nn:.3f}x  identical {same} max|d| {dmax:.2e}", flush=True)
    del x, ws, wts, a, b
    torch.cuda.empty_cache()
