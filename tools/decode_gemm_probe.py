"""Decode-step projection GEMMs at the batch's row count (M = 256 rows at config 2, 16 at config 5): hipBLASLt via
F.linear (default pick, and the decode pins of gemm_tune) against cram_gemm_splitk at several split counts and the
one-pass 4-wave cram_gemm (gemm_w4_kernel; gate/up with its fused SiLU-mul, against hipBLASLt + cram_silu_mul).

Weights are cycled through enough copies to exceed the 256 MB Infinity Cache, so every call streams its weight from
HBM as the decode step does (each layer's weights are read once per step).  Prints one JSON line per (shape, method):
microseconds per call (median over rounds) and the weight stream rate.
Usage (GPU box):  python tools/decode_gemm_probe.py [--model llama3|qwen2] [--M 256]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cram_amd import _lib, gemm_tune, ops  # noqa: E402
from cram_amd.engine import ModelSpec  # noqa: E402


def timeit(fn, copies, reps=5, iters=None):
    iters = iters or max(2 * len(copies), 16)
    for i in range(len(copies)):
        fn(copies[i])
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(iters):
            fn(copies[i % len(copies)])
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / iters)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3")
    ap.add_argument("--M", type=int, default=256)
    ap.add_argument("--hot", action="store_true", help="one weight copy (Infinity-Cache resident) instead of cycling")
    ap.add_argument("--only", default="", help="comma list of shapes")
    args = ap.parse_args()
    sp = ModelSpec.llama3_8b() if args.model == "llama3" else ModelSpec.qwen2_7b()
    dev = torch.device("cuda:0")
    gemm_tune.ensure()
    M, D, F = args.M, sp.hidden, sp.intermediate
    shapes = {"qkv": (sp.q_size + 2 * sp.kv_size, D), "o_proj": (D, sp.q_size), "gate_up": (2 * F, D),
              "down": (D, F), "lm_head": (sp.vocab, D)}
    g = torch.Generator(device=dev).manual_seed(0)
    ws = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    for name, (N, K) in shapes.items():
        wbytes = N * K * 2
        if args.only and name not in args.only.split(","):
            continue
        n_copies = 1 if args.hot else max(2, min(16, -(-(640 << 20) // wbytes)))
        ws_ = [(torch.randn(N, K, generator=g, device=dev) * 0.02).to(torch.bfloat16) for _ in range(n_copies)]
        x = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
        ref = (x.float() @ ws_[0].float().t())
        res = []
        if name == "gate_up":
            base = lambda w: ops.silu_mul(torch.nn.functional.linear(x, w), F)
        else:
            base = lambda w: torch.nn.functional.linear(x, w)
        t = timeit(base, ws_)
        res.append(("hipblaslt_default", t))
        with gemm_tune.pinned(decode=True):
            t = timeit(base, ws_)
        res.append(("hipblaslt_decode_pins", t))
        ntiles = N // 256 if N % 256 == 0 else 0
        if ntiles:
            for s in (1, 2, 4, 7, 8, 14, 16, 28, 32):
                if K % (64 * s) or ops.gemm_splitk_workspace_bytes(M, N, s) > ws.numel():
                    continue
                if ntiles * s > 4096 or (s > 1 and ntiles * s < 64):
                    continue
                epi = ops.GEMM_SILU_MUL_CAT if name == "gate_up" else ops.GEMM_STORE
                fn = lambda w, s=s, epi=epi: ops.gemm_splitk(x, w, s, epi, workspace=ws)
                out = fn(ws_[0])
                if name != "gate_up":
                    err = float((out.float() - ref).abs().max())
                else:
                    err = float((out.float() - ops.silu_mul(ref.to(torch.bfloat16), F).float()).abs().max())
                t = timeit(fn, ws_)
                res.append((f"splitk{s}", t, err))
        if ntiles and K % 64 == 0 and K // 64 >= 2:
            # one-pass cram_gemm on the 4-wave kernel (gemm_w4_kernel); gate/up on the interleaved weight with the
            # fused SiLU-mul epilogue
            prev = _lib.set_knob(_lib.KNOB_GEMM_VARIANT, 1)
            try:
                if name == "gate_up":
                    wil = [ops.interleave_gate_up(w, F) for w in ws_]
                    fn = lambda w: ops.gemm(x, w, ops.GEMM_SILU_MUL)
                    out = fn(wil[0])
                    err = float((out.float() - ops.silu_mul(ref.to(torch.bfloat16), F).float()).abs().max())
                    t = timeit(fn, wil)
                    del wil
                else:
                    fn = lambda w: ops.gemm(x, w)
                    err = float((fn(ws_[0]).float() - ref).abs().max())
                    t = timeit(fn, ws_)
            finally:
                _lib.set_knob(_lib.KNOB_GEMM_VARIANT, prev)
            res.append(("w4", t, err))
        if N % 128 == 0 and K % 64 == 0:
            # cram_gemm_small (128 x 128 tiles, four-deep ring): one pass and K splits; gate/up on the interleaved weight
            # with the fused SiLU-mul
            wil = [ops.interleave_gate_up(w, F) for w in ws_] if name == "gate_up" else None
            for s in (1, 2, 3, 4, 7, 8):
                if K % (64 * s) or ops.gemm_splitk_workspace_bytes(M, N, s) > ws.numel():
                    continue
                if name == "gate_up":
                    fn = lambda w, s=s: ops.gemm_small(x, w, s, ops.GEMM_SILU_MUL, workspace=ws)
                    err = float((fn(wil[0]).float() - ops.silu_mul(ref.to(torch.bfloat16), F).float()).abs().max())
                    t = timeit(fn, wil)
                else:
                    fn = lambda w, s=s: ops.gemm_small(x, w, s, workspace=ws)
                    err = float((fn(ws_[0]).float() - ref).abs().max())
                    t = timeit(fn, ws_)
                res.append((f"sm{s}", t, err))
            del wil
        for r in res:
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "method": r[0], "us": round(r[1], 2),
                              "weight_TBps": round(wbytes / r[1] / 1e6, 3),
                              **({"max_abs_err": r[2]} if len(r) > 2 else {})}), flush=True)
        del ws_


if __name__ == "__main__":
    main()
