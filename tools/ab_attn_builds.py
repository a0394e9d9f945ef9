"""Same-process A/B of the prefill attention kernel between two builds of the library (e.g. the committed HEAD and
the working tree): both .so files are loaded with ctypes and called through the C-ABI on the same inputs,
interleaved rounds, medians (cdna_hip_programming.md §5.4 rule 24).  Also checks the two outputs agree.
  python tools/ab_attn_builds.py tools/ablib/libcram_base.so cram_amd/libcram_attn.so [rounds]
Build the base library with tools/ab_attn_builds.sh <git-rev> (hipcc of that revision's sources, in-tree)."""
import ctypes
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import _lib, ops  # noqa: E402


def load(path):
    lib = ctypes.CDLL(path)
    res, args = _lib.SIGNATURES["cram_attn_prefill"]
    lib.cram_attn_prefill.restype = res
    lib.cram_attn_prefill.argtypes = args
    return lib


def call(lib, q, k, v, out, bias, enable, W):
    B, Hq, Tq, d = q.shape
    S = k.shape[2]
    code = lib.cram_attn_prefill(
        q.data_ptr(), q.stride(0), q.stride(1), q.stride(2), k.data_ptr(), k.stride(0), k.stride(1), k.stride(2),
        v.data_ptr(), v.stride(0), v.stride(1), v.stride(2), out.data_ptr(), out.stride(0), out.stride(2),
        out.stride(1), B, Hq, k.shape[1], Tq, S, d, S - Tq, d ** -0.5,
        bias.data_ptr() if bias is not None else None, bias.stride(0) if bias is not None else 0,
        enable.data_ptr() if enable is not None else None, enable.stride(0) if enable is not None else 0, W, 0,
        torch.cuda.current_stream().cuda_stream)
    assert code == 0, code


def main():
    args = sys.argv[1:]
    rounds = int(args.pop()) if args and args[-1].isdigit() else 7
    paths = args                                   # the first is the base; every other is timed against it
    libs = [load(p) for p in paths]
    dev = torch.device("cuda:0")
    d = 128
    cases = []
    # (B, T, biased, p0): p0 > 0 = the IE sweep's suffix call (T query rows after a p0-token shared prefix of keys)
    for B, T, biased, p0 in [(33, 962, False, 0), (33, 937, False, 25), (1, 962, True, 0), (1, 8300, False, 0),
                             (16, 8300, True, 0)]:
        g = torch.Generator(device=dev).manual_seed(B * T)
        y = torch.randn(B, T + p0, 48 * d, device=dev, generator=g).to(torch.bfloat16)
        q = y[:, p0:, :32 * d].unflatten(-1, (32, d)).transpose(1, 2)
        k = y[..., 32 * d:40 * d].unflatten(-1, (8, d)).transpose(1, 2)
        v = y[..., 40 * d:].unflatten(-1, (8, d)).transpose(1, 2)
        bias = enable = None
        W = 0
        if biased:
            bias = torch.zeros(B, T, device=dev)
            bias[:, 40:400] = -2.3
            bias[:, 500:700] = float("-inf")
            enable = torch.ones(B, 32, dtype=torch.uint8, device=dev)
            W = T
        outs = [torch.empty(B, T, 32, d, device=dev, dtype=torch.bfloat16) for _ in libs]
        cases.append(((B, T, biased, p0), q, k, v, bias, enable, W, outs))
    for name, q, k, v, bias, enable, W, outs in cases:
        for lib, o in zip(libs, outs):
            call(lib, q, k, v, o, bias, enable, W)
        torch.cuda.synchronize()
        for i in range(1, len(libs)):
            dmax = (outs[0].float() - outs[i].float()).abs().max().item()
            print(f"{name}: max |{paths[0].rsplit('/', 1)[-1]} - {paths[i].rsplit('/', 1)[-1]}| = {dmax:.3e}",
                  flush=True)
    res = {(i, c[0]): [] for i in range(len(libs)) for c in cases}
    for _ in range(rounds):
        for i, lib in enumerate(libs):
            for name, q, k, v, bias, enable, W, outs in cases:
                for _ in range(2):
                    call(lib, q, k, v, outs[i], bias, enable, W)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    call(lib, q, k, v, outs[i], bias, enable, W)
                e1.record()
                torch.cuda.synchronize()
                res[(i, name)].append(e0.elapsed_time(e1) / 10)
    for name, q, *_ in cases:
        B, T, _b, p0 = name
        fl, _ = ops.prefill_work(B, 32, 8, T, T + p0, d, p0)
        ms = [statistics.median(res[(i, name)]) for i in range(len(libs))]
        print(f"{str(name):22s} " + "  ".join(
            f"{paths[i].rsplit('/', 1)[-1]} {ms[i]:.3f} ms {fl / ms[i] / 1e9:6.0f} TF ({fl / ms[i] / 2.5e12:.3f})"
            + ("" if i == 0 else f" {ms[0] / ms[i]:.3f}x") for i in range(len(libs))), flush=True)


if __name__ == "__main__":
    main()
