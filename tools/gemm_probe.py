"""Same-process A/B of cram_gemm (hand-written MFMA GEMM) against hipBLASLt (F.linear) at the IE sweep's shapes.

Interleaved rounds, medians (cdna_hip_programming.md §5.4 rule 24); uniform random operands (rule 25).
  python tools/gemm_probe.py [M] [rounds]
Shapes (Llama-3-8B, M = sweep rows): q/k/v N 6144 K 4096, o_proj N 4096 K 4096, gate/up N 28672 K 4096 (alone,
and with the MLP activation: hipBLASLt + cram_silu_mul vs cram_gemm's fused SiLU-mul epilogue), down N 4096 K 14336.
"""
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import ops  # noqa: E402


def timeit(fn, iters=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 29184
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    torch.backends.cuda.preferred_blas_library("hipblaslt")
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    D, F = 4096, 14336
    x = (torch.rand(M, D, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    xf = (torch.rand(M, F, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    W = {n: ((torch.rand(n, D, device=dev, generator=g) * 2 - 1) * D ** -0.5).to(torch.bfloat16)
         for n in (6144, 4096, 2 * F)}
    wgu = W[2 * F]
    wil = ops.interleave_gate_up(wgu, F)
    wd = ((torch.rand(4096, F, device=dev, generator=g) * 2 - 1) * F ** -0.5).to(torch.bfloat16)
    cases = {
        "qkv  lt": (lambda: torch.nn.functional.linear(x, W[6144]), 2 * M * 6144 * D),
        "qkv  cr": (lambda: ops.gemm(x, W[6144]), 2 * M * 6144 * D),
        "o    lt": (lambda: torch.nn.functional.linear(x, W[4096]), 2 * M * 4096 * D),
        "o    cr": (lambda: ops.gemm(x, W[4096]), 2 * M * 4096 * D),
        "gu   lt": (lambda: torch.nn.functional.linear(x, wgu), 2 * M * 2 * F * D),
        "gu   cr": (lambda: ops.gemm(x, wgu), 2 * M * 2 * F * D),
        "gu+act lt+silu": (lambda: ops.silu_mul(torch.nn.functional.linear(x, wgu), F), 2 * M * 2 * F * D),
        "gu+act cr fused": (lambda: ops.gemm(x, wil, ops.GEMM_SILU_MUL), 2 * M * 2 * F * D),
        "down lt": (lambda: torch.nn.functional.linear(xf, wd), 2 * M * 4096 * F),
        "down cr": (lambda: ops.gemm(xf, wd), 2 * M * 4096 * F),
    }
    # correctness spot check before timing
    a = ops.gemm(x, W[4096])
    b = torch.nn.functional.linear(x, W[4096])
    torch.cuda.synchronize()
    print(f"M={M}: cram vs hipBLASLt o_proj max |diff| {(a.float() - b.float()).abs().max().item():.3e}", flush=True)
    for fn, _ in cases.values():        # warm-up (clocks, allocator, kernel selection)
        timeit(fn, 2)
    res = {k: [] for k in cases}
    t0 = time.time()
    for r in range(rounds):
        for k, (fn, _) in cases.items():
            res[k].append(timeit(fn))
    for k, (fn, fl) in cases.items():
        med = statistics.median(res[k])
        print(f"{k:18s} median {med:8.3f} ms  min {min(res[k]):8.3f}  {fl / med / 1e9:7.1f} TFLOP/s", flush=True)
    for a_, b_ in [("qkv  lt", "qkv  cr"), ("o    lt", "o    cr"), ("gu   lt", "gu   cr"),
                   ("gu+act lt+silu", "gu+act cr fused"), ("down lt", "down cr")]:
        print(f"{b_:18s} / {a_:18s} speed {statistics.median(res[a_]) / statistics.median(res[b_]):.3f}x")
    print(f"({time.time() - t0:.1f}s)")


if __name__ == "__main__":
    main()
