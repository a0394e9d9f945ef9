"""Same-process A/B of the default hipBLASLt pick vs the pinned solutions (cram_amd/gemm_tune.py) across the row
counts the sweep produces.  Interleaved rounds, median ms per Llama-3-8B layer (the four projection GEMMs).

    python tools/pinned_gemm_probe.py [M ...]
"""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cram_amd import gemm_tune  # noqa: E402

dev = torch.device("cuda:0")
Ms = [int(a) for a in sys.argv[1:]] or [8192, 16384, 23040, 26112, 29184, 32768]
shapes = [(4096, 6144), (4096, 4096), (4096, 28672), (14336, 4096)]
print("pinned:", gemm_tune.install(gemm_tune.sweep_rows()), flush=True)
torch.cuda.tunable.enable(True)              # pins act while TunableOp is on (gemm_tune.pinned)
torch.cuda.tunable.tuning_enable(False)
W = [(K, N, (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)) for K, N in shapes]
X = {M: {K: torch.randn(M, K, device=dev).to(torch.bfloat16) for K in (4096, 14336)} for M in Ms}


def layer_ms(M, pinned):
    torch.cuda.tunable.enable(pinned)
    out = []
    for K, N, w in W:
        x = X[M][K]
        for _ in range(2):
            F.linear(x, w)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(8):
            F.linear(x, w)
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / 8)
    return out


for M in Ms:
    res = {False: [], True: []}
    for rnd in range(5):
        for pinned in (False, True):
            res[pinned].append(layer_ms(M, pinned))
    med = {p: [statistics.median(r[i] for r in res[p]) for i in range(len(shapes))] for p in res}
    print(f"M={M}: default {sum(med[False]):.3f} ms [" + " ".join(f"{x:.3f}" for x in med[False]) + "]  pinned "
          f"{sum(med[True]):.3f} ms [" + " ".join(f"{x:.3f}" for x in med[True]) + f"]  "
          f"-> {sum(med[False]) / sum(med[True]):.3f}x", flush=True)
