"""Per-layer GEMM time of Llama-3-8B's four projections as a function of the row count M (with the pinned solutions
of cram_amd/gemm_tune.py), over the sweep's range, for choosing padded row counts (data/gemm_rows.json).
Rounds are outer and row counts inner, so clock drift spreads over all M; median per M.

    python tools/gemm_rows_sweep.py [lo hi step rounds] > gpurun_out/rows.json
"""
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cram_amd import gemm_tune  # noqa: E402

lo, hi, step, rounds = (int(a) for a in (sys.argv[1:5] if len(sys.argv) >= 5 else (16384, 40960, 256, 5)))
dev = torch.device("cuda:0")
pinned = gemm_tune.install(gemm_tune.sweep_rows())
torch.cuda.tunable.enable(True)              # pins act while TunableOp is on (gemm_tune.pinned)
torch.cuda.tunable.tuning_enable(False)
shapes = [(4096, 6144), (4096, 4096), (4096, 28672), (14336, 4096)]
W = [(K, (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)) for K, N in shapes]
X = {K: torch.randn(hi, K, device=dev).to(torch.bfloat16) for K in (4096, 14336)}
Ms = list(range(lo, hi + 1, step))
res = {M: [] for M in Ms}
for rnd in range(rounds):
    for M in Ms:
        tot = 0.0
        for K, w in W:
            x = X[K][:M]
            F.linear(x, w)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(4):
                F.linear(x, w)
            e.record()
            torch.cuda.synchronize()
            tot += s.elapsed_time(e) / 4
        res[M].append(tot)
    print(f"round {rnd} done", file=sys.stderr, flush=True)
print(json.dumps({"pinned": pinned, "shapes_NK": [[N, K] for K, N in shapes],
                  "layer_gemm_ms": {str(M): round(statistics.median(v), 4) for M, v in res.items()}}))
