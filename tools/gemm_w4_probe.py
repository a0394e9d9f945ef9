"""Same-process A/B of the projection GEMMs at the IE sweep's shapes: cram_gemm on the 4-wave kernel (gemm_w4_kernel,
knob CRAM_KNOB_GEMM_VARIANT = 1), on the 8-wave kernel (0), and hipBLASLt (F.linear) with its default pick and inside
gemm_tune.pinned() (the sweep's TunableOp solutions for q/k/v and o_proj).  Every cram result is first checked
against the float32 product (each element within 1 bf16 ulp + 2^-22 sum|xw|).

  python tools/gemm_w4_probe.py [M] [rounds]
Interleaved rounds, medians; uniform random operands (cdna_hip_programming.md §5.4 rules 24, 25).
"""
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import _lib, gemm_tune, ops  # noqa: E402


def timeit(fn, iters=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def variant(v, fn):
    def run():
        prev = _lib.set_knob(_lib.KNOB_GEMM_VARIANT, v)
        try:
            return fn()
        finally:
            _lib.set_knob(_lib.KNOB_GEMM_VARIANT, prev)
    return run


def pinned(fn):
    def run():
        with gemm_tune.pinned():
            return fn()
    return run


def check(name, got, x, w, silu_F=None):
    ref = x.float() @ w.float().t()
    bound = x.float().abs() @ w.float().abs().t()
    if silu_F is not None:
        g, u = ref[:, :silu_F].to(torch.bfloat16).float(), ref[:, silu_F:].to(torch.bfloat16).float()
        ref = (torch.nn.functional.silu(g).to(torch.bfloat16).float() * u)
        bound = bound[:, :silu_F] + bound[:, silu_F:]
    err = (got.float() - ref).abs()
    ulp = ref.abs() * 2.0 ** -8
    bad = (err > ulp + 2.0 ** -22 * bound + (1e-2 if silu_F else 0)).sum().item()
    print(f"{name:22s} max |err| {err.max().item():.3e}  elements outside the bar: {bad}", flush=True)
    return bad == 0


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 29184
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    torch.backends.cuda.preferred_blas_library("hipblaslt")
    gemm_tune.ensure()
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
    ok = True
    rows = slice(0, 2048)
    for nm, xx, ww in (("qkv", x, W[6144]), ("o", x, W[4096]), ("down", xf, wd)):
        ok &= check(f"{nm} w4", variant(1, lambda: ops.gemm(xx, ww))()[rows], xx[rows], ww)
    ok &= check("gu+act w4 fused", variant(1, lambda: ops.gemm(x, wil, ops.GEMM_SILU_MUL))()[rows], x[rows], wgu,
                silu_F=F)
    tail = x[:M - 77]                                   # a ragged last row tile
    ok &= check("o w4 ragged M", variant(1, lambda: ops.gemm(tail, W[4096]))()[-1024:], tail[-1024:], W[4096])
    print("correct" if ok else "MISMATCH", flush=True)
    if not ok:
        sys.exit(1)
    cases = {}
    for nm, xx, ww, fl in (("qkv", x, W[6144], 2 * M * 6144 * D), ("o", x, W[4096], 2 * M * 4096 * D),
                           ("gu", x, wgu, 2 * M * 2 * F * D), ("down", xf, wd, 2 * M * 4096 * F)):
        cases[f"{nm} lt"] = (lambda xx=xx, ww=ww: torch.nn.functional.linear(xx, ww), fl)
        cases[f"{nm} lt-pinned"] = (pinned(lambda xx=xx, ww=ww: torch.nn.functional.linear(xx, ww)), fl)
        cases[f"{nm} w4"] = (variant(1, lambda xx=xx, ww=ww: ops.gemm(xx, ww)), fl)
        cases[f"{nm} 8w"] = (variant(0, lambda xx=xx, ww=ww: ops.gemm(xx, ww)), fl)
    cases["gu+act lt+silu"] = (lambda: ops.silu_mul(torch.nn.functional.linear(x, wgu), F), 2 * M * 2 * F * D)
    cases["gu+act w4 fused"] = (variant(1, lambda: ops.gemm(x, wil, ops.GEMM_SILU_MUL)), 2 * M * 2 * F * D)
    for fn, _ in cases.values():
        timeit(fn, 2)
    res = {k: [] for k in cases}
    t0 = time.time()
    for _ in range(rounds):
        for k, (fn, _) in cases.items():
            res[k].append(timeit(fn))
    for k, (fn, fl) in cases.items():
        med = statistics.median(res[k])
        print(f"{k:18s} median {med:8.3f} ms  min {min(res[k]):8.3f}  {fl / med / 1e12:7.1f} TFLOP/s", flush=True)
    for nm in ("qkv", "o", "gu", "down"):
        best_lt = min(statistics.median(res[f"{nm} lt"]), statistics.median(res[f"{nm} lt-pinned"]))
        print(f"{nm:5s} w4 / best hipBLASLt {best_lt / statistics.median(res[f'{nm} w4']):.3f}x   "
              f"8w / best hipBLASLt {best_lt / statistics.median(res[f'{nm} 8w']):.3f}x")
    print(f"gu+act w4 fused / hipBLASLt + silu_mul "
          f"{statistics.median(res['gu+act lt+silu']) / statistics.median(res['gu+act w4 fused']):.3f}x")
    print(f"({time.time() - t0:.1f}s)")


if __name__ == "__main__":
    main()
