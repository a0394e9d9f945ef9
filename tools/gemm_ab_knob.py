"""Same-process A/B of cram_gemm under several CRAM_KNOB_GEMM_VARIANT values (kernel / tile-order variants) against
hipBLASLt (default pick and the sweep's pinned solutions) at the sweep's projection shapes.  Interleaved rounds,
medians, uniform random operands.   python tools/gemm_ab_knob.py M rounds knob [knob ...]"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import _lib, gemm_tune, ops  # noqa: E402


def timeit(fn, iters=4):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


M, rounds = int(sys.argv[1]), int(sys.argv[2])
knobs = [int(k) for k in sys.argv[3:]]
torch.backends.cuda.preferred_blas_library("hipblaslt")
gemm_tune.ensure()
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
D, F = 4096, 14336
x = (torch.rand(M, D, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
xf = (torch.rand(M, F, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
W = {n: ((torch.rand(n, D, device=dev, generator=g) * 2 - 1) * D ** -0.5).to(torch.bfloat16) for n in (6144, 4096, 2 * F)}
wil = ops.interleave_gate_up(W[2 * F], F)
wd = ((torch.rand(4096, F, device=dev, generator=g) * 2 - 1) * F ** -0.5).to(torch.bfloat16)
shapes = {"qkv": (x, W[6144], 2 * M * 6144 * D), "o": (x, W[4096], 2 * M * 4096 * D),
          "gu": (x, W[2 * F], 2 * M * 2 * F * D), "down": (xf, wd, 2 * M * 4096 * F)}


def with_knob(v, fn):
    def run():
        prev = _lib.set_knob(_lib.KNOB_GEMM_VARIANT, v)
        try:
            fn()
        finally:
            _lib.set_knob(_lib.KNOB_GEMM_VARIANT, prev)
    return run


def pinned(fn):
    def run():
        with gemm_tune.pinned():
            fn()
    return run


cases = {}
ref = {}
for nm, (xx, ww, fl) in shapes.items():
    cases[(nm, "lt")] = (lambda xx=xx, ww=ww: torch.nn.functional.linear(xx, ww), fl)
    cases[(nm, "ltpin")] = (pinned(lambda xx=xx, ww=ww: torch.nn.functional.linear(xx, ww)), fl)
    for k in knobs:
        cases[(nm, f"k{k}")] = (with_knob(k, lambda xx=xx, ww=ww: ops.gemm(xx, ww)), fl)
    ref[nm] = torch.nn.functional.linear(xx[:512], ww).float()
cases[("gu+act", "lt+silu")] = (lambda: ops.silu_mul(torch.nn.functional.linear(x, W[2 * F]), F), shapes["gu"][2])
for k in knobs:
    cases[("gu+act", f"k{k}")] = (with_knob(k, lambda: ops.gemm(x, wil, ops.GEMM_SILU_MUL)), shapes["gu"][2])
for k in knobs:                                          # every variant agrees with hipBLASLt within bf16 rounding
    for nm, (xx, ww, _) in shapes.items():
        prev = _lib.set_knob(_lib.KNOB_GEMM_VARIANT, k)
        d = (ops.gemm(xx[:512], ww).float() - ref[nm]).abs().max().item()
        _lib.set_knob(_lib.KNOB_GEMM_VARIANT, prev)
        assert d < 2e-2, (k, nm, d)
for fn, _ in cases.values():
    timeit(fn, 2)
res = {k: [] for k in cases}
for _ in range(rounds):
    for k, (fn, _) in cases.items():
        res[k].append(timeit(fn))
for nm in list(shapes) + ["gu+act"]:
    base = min(statistics.median(res[(nm, b)]) for b in ("lt", "ltpin") if (nm, b) in res) if nm != "gu+act" \
        else statistics.median(res[(nm, "lt+silu")])
    row = []
    for (n2, v), t in res.items():
        if n2 == nm:
            med = statistics.median(t)
            row.append(f"{v} {med:.3f} ms ({base / med:.3f}x)")
    print(f"{nm:7s} " + " | ".join(row), flush=True)
