"""Decode-step GEMMs (M = batch rows, weight-streaming): hipBLASLt's default heuristic pick vs PyTorch TunableOp's
tuned pick, same process, interleaved rounds, medians; writes the tuned solution names per (N, K, M).

At M = 256 the decode step's projections read every weight once per step, so their bound is HBM (weights / 8 TB/s)
or the matrix cores (2 M N K / 2.5 PF), whichever is larger; the rocprofv3 summary of the decode leg showed the
default picks at 1.3-3.4 TB/s (`profiles/r02/s4_decode_leg_kernel_stats.csv`).

    python tools/tune_decode_gemms.py [--models llama3-8b,qwen2-7b] [--m 256,16] [--out gpurun_out/decode_gemms.json]
"""
import argparse
import json
import os
import statistics

import torch
import torch.nn.functional as F

SHAPES = {   # (K, N) of F.linear(x [M, K], w [N, K]): q/k/v, o_proj, gate/up, down, lm_head
    "llama3-8b": [(4096, 6144), (4096, 4096), (4096, 28672), (14336, 4096), (4096, 128256)],
    "qwen2-7b": [(3584, 3584), (3584, 37888), (18944, 3584), (3584, 152064)],   # q/k/v has a bias: not here
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="llama3-8b,qwen2-7b")
    ap.add_argument("--m", default="256,16")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--out", default="gpurun_out/decode_gemms.json")
    ap.add_argument("--tune-ms", type=int, default=300)
    ap.add_argument("--rotate-mb", type=int, default=1024)
    ap.add_argument("--cold-mb", type=int, default=768, help="weight copies cycled in the timing loop span this (cold MALL)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    tun = torch.cuda.tunable
    tun.set_filename(os.path.join(os.path.dirname(a.out) or ".", "tunableop_decode%d.csv"))
    tun.set_max_tuning_duration(a.tune_ms)
    tun.set_max_tuning_iterations(100)
    if hasattr(tun, "set_rotating_buffer_size"):
        tun.set_rotating_buffer_size(a.rotate_mb)      # candidates timed with cold caches, as in a decode step
    cases = []
    for model in a.models.split(","):
        for K, N in SHAPES[model]:
            nc = min(16, max(2, -(-a.cold_mb * 2**20 // (N * K * 2))))   # copies spanning >= cold_mb
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(nc)]
            for M in (int(x) for x in a.m.split(",")):
                cases.append((model, M, K, N, torch.randn(M, K, device=dev).to(torch.bfloat16), ws))

    def timed(x, ws):
        # the step streams 15 GB of distinct weights: cycling copies keeps a 50-250 MB weight out of the 256 MB MALL
        for w in ws:
            F.linear(x, w)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(20):
            F.linear(x, ws[i % len(ws)])
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / 20

    tun.enable(True)
    tun.tuning_enable(True)
    for *_, x, ws in cases:          # one call per shape tunes it
        F.linear(x, ws[0])
    torch.cuda.synchronize()
    results = {r[1]: r[2] for r in tun.get_results()}
    tun.tuning_enable(False)
    res = {(i, on): [] for i in range(len(cases)) for on in (False, True)}
    for _ in range(a.rounds):
        for on in (False, True):
            tun.enable(on)
            for i, (*_, x, ws) in enumerate(cases):
                res[(i, on)].append(timed(x, ws))
    tun.enable(False)
    out = {"validators": {str(k): str(v) for k, v in tun.get_validators()}, "cases": []}
    for i, (model, M, K, N, x, _) in enumerate(cases):
        d0, d1 = statistics.median(res[(i, False)]), statistics.median(res[(i, True)])
        sig = f"tn_{N}_{M}_{K}_ld_{K}_{K}_{N}"
        gb = (N * K + M * K + M * N) * 2 / 1e9
        row = {"model": model, "M": M, "K": K, "N": N, "default_ms": d0, "tuned_ms": d1, "speedup": d0 / d1,
               "default_tbs": gb / d0, "tuned_tbs": gb / d1, "solution": results.get(sig)}
        out["cases"].append(row)
        print(f"{model:10s} M={M:4d} K={K:5d} N={N:6d}  default {d0 * 1e3:7.1f} us ({gb / d0:4.2f} TB/s)  "
              f"tuned {d1 * 1e3:7.1f} us ({gb / d1:4.2f} TB/s)  {d0 / d1:5.2f}x  {row['solution']}", flush=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
