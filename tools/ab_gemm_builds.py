"""Same-process A/B of the projection GEMM (gemm_w4_kernel, every epilogue) between two builds of the library: both
.so files are loaded with ctypes and called through the C-ABI on the same inputs at the IE sweep's shapes (M rows of
the Llama-3-8B suffix batch), interleaved rounds, medians (cdna_hip_programming.md §5.4 rule 24; uniform random
operands, rule 25).  Also reports how the two builds' outputs differ (bit-equal elements, max ulp distance).

  python tools/ab_gemm_builds.py BASE.so NEW.so [M] [rounds]
Build BASE with  OUTDIR=tools/abbase bash tools/ab_attn_builds.sh <git-rev>."""
import ctypes
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import _lib, gemm_tune, ops  # noqa: E402

NAMES = ("cram_gemm", "cram_gemm_residual", "cram_gemm_rope")


def load(path):
    lib = ctypes.CDLL(path)
    for n in NAMES:
        res, args = _lib.SIGNATURES[n]
        getattr(lib, n).restype = res
        getattr(lib, n).argtypes = args
    return lib


def timeit(fn, iters=4):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def ulps(a, b):
    """Largest distance in bf16 ulps between two bf16 tensors (sign-magnitude order)."""
    ia = a.view(torch.int16).int()
    ib = b.view(torch.int16).int()
    oa = torch.where(ia < 0, -(ia & 0x7FFF), ia)
    ob = torch.where(ib < 0, -(ib & 0x7FFF), ib)
    return int((oa - ob).abs().max())


def main():
    base, new = sys.argv[1], sys.argv[2]
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 29184
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 7
    libs = {"base": load(base), "new": load(new)}
    torch.backends.cuda.preferred_blas_library("hipblaslt")
    gemm_tune.ensure()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    D, F, NQKV, T, p0 = 4096, 14336, 6144, 912, 25
    bf = torch.bfloat16
    x = (torch.rand(M, D, device=dev, generator=g) * 2 - 1).to(bf)
    xf = (torch.rand(M, F, device=dev, generator=g) * 2 - 1).to(bf)
    w = {n: ((torch.rand(n, D, device=dev, generator=g) * 2 - 1) * D ** -0.5).to(bf) for n in (NQKV, D, 2 * F)}
    wil = ops.interleave_gate_up(w[2 * F], F)
    wd = ((torch.rand(D, F, device=dev, generator=g) * 2 - 1) * F ** -0.5).to(bf)
    res = torch.randn(M, D, device=dev, generator=g).to(bf)
    B = M // T
    cos = torch.randn(p0 + T, 128, device=dev, generator=g).to(bf)
    sin = torch.randn(p0 + T, 128, device=dev, generator=g).to(bf)
    kout = {k: torch.empty(B, p0 + T, 8, 128, device=dev, dtype=bf) for k in libs}
    vout = {k: torch.empty_like(kout[k]) for k in libs}
    outs = {}

    def gemm(k, a, wt, epi, n_out):
        o = outs.setdefault((k, "g", epi, wt.shape[0], a.shape[1]), torch.empty(M, n_out, device=dev, dtype=bf))
        return lambda: _lib.check(libs[k].cram_gemm(a.data_ptr(), a.stride(0), wt.data_ptr(), wt.stride(0), o.data_ptr(),
                                                    o.stride(0), M, wt.shape[0], a.shape[1], epi, ops.DTYPES[bf], st),
                                  "cram_gemm")

    def resid(k, a, wt):
        o = outs.setdefault((k, "r", wt.shape[1]), torch.empty(M, D, device=dev, dtype=bf))
        return lambda: _lib.check(libs[k].cram_gemm_residual(a.data_ptr(), a.stride(0), wt.data_ptr(), wt.stride(0),
                                                             res.data_ptr(), res.stride(0), o.data_ptr(), o.stride(0),
                                                             M, D, a.shape[1], ops.DTYPES[bf], st), "residual")

    def rope(k):
        o = outs.setdefault((k, "rope"), torch.empty(M, NQKV, device=dev, dtype=bf))
        kc, vc = kout[k], vout[k]
        rows = B * T
        return lambda: _lib.check(libs[k].cram_gemm_rope(
            x.data_ptr(), x.stride(0), w[NQKV].data_ptr(), w[NQKV].stride(0), None, o.data_ptr(), o.stride(0), M, D,
            rows, T, 32, 8, 128, cos.data_ptr(), sin.data_ptr(), cos.stride(0), None, p0, kc.data_ptr(), vc.data_ptr(),
            kc.stride(0), kc.stride(2), kc.stride(1), p0, None, 0, ops.DTYPES[bf], st), "rope")

    cases = {
        "gate/up + SiLU-mul": (lambda k: gemm(k, x, wil, ops.GEMM_SILU_MUL, F), 2.0 * M * 2 * F * D),
        "gate/up store": (lambda k: gemm(k, x, w[2 * F], ops.GEMM_STORE, 2 * F), 2.0 * M * 2 * F * D),
        "o_proj + residual": (lambda k: resid(k, x, w[D]), 2.0 * M * D * D),
        "down + residual": (lambda k: resid(k, xf, wd), 2.0 * M * D * F),
        "q/k/v + RoPE": (lambda k: rope(k), 2.0 * M * NQKV * D),
    }
    fns = {(c, k): f(k) for c, (f, _) in cases.items() for k in libs}
    for fn in fns.values():
        fn()
    torch.cuda.synchronize()
    times = {key: [] for key in fns}
    for _ in range(rounds):
        for key, fn in fns.items():
            times[key].append(timeit(fn))
    print(f"M = {M}, {rounds} interleaved rounds, medians (min) in ms; TFLOP/s of the median")
    for c, (_, fl) in cases.items():
        b, n = statistics.median(times[(c, "base")]), statistics.median(times[(c, "new")])
        print(f"  {c:20s} base {b:7.3f} ({min(times[(c, 'base')]):.3f})  new {n:7.3f} ({min(times[(c, 'new')]):.3f})"
              f"  new/base speed {b / n:6.3f}x   {fl / n / 1e9:7.1f} TFLOP/s")
    # output agreement of the two builds (each case's result from its last launch)
    for kind in {k[1:] for k in outs if k[0] == "base"}:
        a, b = outs[("base",) + kind], outs[("new",) + kind]
        nd = int((a != b).sum())
        print(f"  outputs {str(kind):34s} {nd} of {a.numel()} elements differ, max ulp {ulps(a, b)}")
    eqk = float((kout['base'][:, p0:] == kout['new'][:, p0:]).float().mean())
    eqv = float((vout['base'][:, p0:] == vout['new'][:, p0:]).float().mean())
    print(f"  rope k / v written behind the prefix: bit-equal {eqk:.6f} / {eqv:.6f}")


if __name__ == "__main__":
    main()
