"""Fixed vs per-K-tile cost of cram_gemm's 4-wave kernel and hipBLASLt: the same N x M output at K = 2048 / 4096 /
8192 (t(K) = fixed + K * per_k, least squares), the gate/up width N = 28672 at M = 29184.  Same process, interleaved
rounds, medians.   python tools/gemm_kscale_probe.py [M] [N]"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import _lib, ops  # noqa: E402


def timeit(fn, iters=4):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


M = int(sys.argv[1]) if len(sys.argv) > 1 else 29184
N = int(sys.argv[2]) if len(sys.argv) > 2 else 28672
torch.backends.cuda.preferred_blas_library("hipblaslt")
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
Ks = (2048, 4096, 8192)
X = {K: (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16) for K in Ks}
W = {K: ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * K ** -0.5).to(torch.bfloat16) for K in Ks}
_lib.set_knob(_lib.KNOB_GEMM_VARIANT, 1)
cases = {}
for K in Ks:
    cases[("lt", K)] = lambda K=K: torch.nn.functional.linear(X[K], W[K])
    cases[("w4", K)] = lambda K=K: ops.gemm(X[K], W[K])
for fn in cases.values():
    timeit(fn, 2)
res = {k: [] for k in cases}
for _ in range(5):
    for k, fn in cases.items():
        res[k].append(timeit(fn))
for impl in ("lt", "w4"):
    t = [statistics.median(res[(impl, K)]) for K in Ks]
    n = len(Ks)
    mk, mt = sum(Ks) / n, sum(t) / n
    b = sum((k - mk) * (y - mt) for k, y in zip(Ks, t)) / sum((k - mk) ** 2 for k in Ks)
    a = mt - b * mk
    print(f"{impl}: " + "  ".join(f"K={K}: {y:.3f} ms ({2 * M * N * K / y / 1e9:.0f} TF)" for K, y in zip(Ks, t))
          + f"  -> fixed {a:.3f} ms + {b * 4096:.3f} ms per 4096 of K")
