"""Same-process A/B of hipBLASLt's default heuristic pick vs PyTorch TunableOp's tuned pick for the IE sweep's
four GEMM shapes (Llama-3-8B, M = 33 x T rows).  Interleaved rounds, median ms per shape.

    python tools/tunable_probe.py [M]
"""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

dev = torch.device("cuda:0")
M = int(sys.argv[1]) if len(sys.argv) > 1 else 29184
shapes = [(4096, 6144), (4096, 4096), (4096, 28672), (14336, 4096)]
os.makedirs("gpurun_out", exist_ok=True)
torch.cuda.tunable.set_filename("gpurun_out/tunableop_results%d.csv")
torch.cuda.tunable.set_max_tuning_duration(200)
torch.cuda.tunable.set_max_tuning_iterations(40)
ops = []
for K, N in shapes:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    ops.append((K, N, x, w))


def run(tuned):
    torch.cuda.tunable.enable(tuned)
    torch.cuda.tunable.tuning_enable(tuned)
    out = []
    for K, N, x, w in ops:
        for _ in range(3):
            F.linear(x, w)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            F.linear(x, w)
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / 10)
    return out


run(True)            # tunes every shape once
print("tuned results:", torch.cuda.tunable.get_results(), flush=True)
res = {False: [], True: []}
for rnd in range(6):
    for tuned in (False, True):
        res[tuned].append(run(tuned))
for tuned in (False, True):
    med = [statistics.median(r[i] for r in res[tuned]) for i in range(len(shapes))]
    tf = [2 * M * K * N / ms / 1e9 for (K, N), ms in zip(shapes, med)]
    print(f"{'tunableop' if tuned else 'default  '} M={M}: " + " | ".join(
        f"K{K} N{N} {ms:.3f} ms {t:.0f} TF" for (K, N), ms, t in zip(shapes, med, tf)) + f" | total {sum(med):.3f} ms")
