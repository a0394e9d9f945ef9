"""GEMM microbench for the IE-sweep shapes: hipBLASLt vs rocBLAS, NT vs NN weight layout."""
import sys
import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")
M = int(sys.argv[1]) if len(sys.argv) > 1 else 33 * 962
shapes = [(4096, 6144), (4096, 4096), (4096, 28672), (14336, 4096)]
print("preferred", torch.backends.cuda.preferred_blas_library())


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for lib in ("hipblaslt", "hipblas", "ck"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as ex:
        print(lib, "unavailable", ex)
        continue
    tot = 0
    for K, N in shapes:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        wt = w.t().contiguous()
        ms = bench(lambda: F.linear(x, w))
        ms2 = bench(lambda: x @ wt)
        fl = 2 * M * K * N
        tot += ms
        print(f"{lib:9s} M={M} K={K} N={N}: NT {ms:.3f} ms {fl/ms/1e9:.0f} TF | NN {ms2:.3f} ms {fl/ms2/1e9:.0f} TF")
    print(lib, "layer total NT ms", round(tot, 3))
