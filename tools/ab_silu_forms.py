"""The SiLU forms of cram_silu.inc (CRAM_SILU_FORM 0 IEEE, 1 hardware exp2 / rcp, 2 expf + rcp + one Newton step,
3 two-term exp2 + rcp + Newton) side by side in one process: cram_silu_mul against torch's silu on the bf16 test
inputs of tests/test_kernels_gpu.py (2 * randn, F = 14336 / 18944), and the fused gate/up + SiLU-mul GEMM at the
sweep's shape (M = 29,184) timed interleaved.
  python tools/ab_silu_forms.py   (after bash tools/ab_silu_forms.sh)"""
import ctypes
import glob
import os
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import _lib, ops  # noqa: E402


def load(path):
    lib = ctypes.CDLL(path)
    for n in ("cram_silu_mul", "cram_gemm"):
        res, args = _lib.SIGNATURES[n]
        getattr(lib, n).restype = res
        getattr(lib, n).argtypes = args
    return lib


def ulp16(a, b):
    ia, ib = a.view(torch.int16).int(), b.view(torch.int16).int()
    oa = torch.where(ia < 0, -(ia & 0x7FFF), ia)
    ob = torch.where(ib < 0, -(ib & 0x7FFF), ib)
    return (oa - ob).abs()


def main():
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "absilu")
    libs = {os.path.basename(p)[len("libcram_f"):-3]: load(p) for p in sorted(glob.glob(os.path.join(root, "libcram_f*.so")))}
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    for F in (14336, 18944):
        gu = (2 * torch.randn(3, 50, 2 * F, device=dev, generator=g)).to(bf)
        ref = torch.nn.functional.silu(gu[..., :F]) * gu[..., F:]
        for k, L in libs.items():
            y = torch.empty_like(ref)
            _lib.check(L.cram_silu_mul(gu.data_ptr(), 2 * F, y.data_ptr(), F, 150, F, 0, st), "silu_mul")
            torch.cuda.synchronize()
            u = ulp16(y, ref)
            print(f"F={F} form {k}: max ulp {int(u.max())}, exact {float((u == 0).float().mean()):.6f}, "
                  f"2-ulp {int((u >= 2).sum())}")
    M, D, Fm = 29184, 4096, 14336
    x = (torch.rand(M, D, device=dev, generator=g) * 2 - 1).to(bf)
    w = ((torch.rand(2 * Fm, D, device=dev, generator=g) * 2 - 1) * D ** -0.5).to(bf)
    wil = ops.interleave_gate_up(w, Fm)
    outs = {k: torch.empty(M, Fm, device=dev, dtype=bf) for k in libs}

    def run(k):
        _lib.check(libs[k].cram_gemm(x.data_ptr(), D, wil.data_ptr(), D, outs[k].data_ptr(), Fm, M, 2 * Fm, D,
                                     ops.GEMM_SILU_MUL, 0, st), "gemm")

    times = {k: [] for k in libs}
    for k in libs:
        run(k)
    torch.cuda.synchronize()
    for _ in range(5):
        for k in libs:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(4):
                run(k)
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / 4)
    for k in libs:
        d = int((outs[k] != outs["0"]).sum()) if "0" in outs else -1
        print(f"gate/up + SiLU-mul M={M}: form {k} {statistics.median(times[k]):.3f} ms; {d} outputs differ from form 0")


if __name__ == "__main__":
    main()
