"""Per-layer projection-GEMM time of Llama-3-8B as a function of the row count M, over the sweep's range, for
choosing padded row counts (data/gemm_rows.json).  Times the engine's own suffix-layer calls: q/k/v with the RoPE
epilogue (cram_gemm_rope), o_proj with the residual epilogue (CrAMEngine._gemm_residual: tail split included),
gate/up with the SiLU-mul epilogue, down_proj with the residual epilogue -- so the table follows whatever kernels
and tail handling the engine runs.  Rounds are outer and row counts inner, so clock drift spreads over all M;
median per M.

    python tools/gemm_rows_sweep.py [lo hi step rounds [no-tail]] > gpurun_out/rows.json

no-tail: o_proj / down_proj without the split-K tail (engine.no_tail_split: the IE sweep's row-exact mode), the table
engine.padded_rows uses for those batches ("layer_gemm_ms_no_tail").
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cram_amd import engine as E, ops  # noqa: E402

lo, hi, step, rounds = (int(a) for a in (sys.argv[1:5] if len(sys.argv) >= 5 else (16384, 40960, 256, 5)))
NO_TAIL = len(sys.argv) > 5 and sys.argv[5] == "no-tail"
dev = torch.device("cuda:0")
sp = E.ModelSpec(1, 4096, 32, 8, 128, 14336, 1000, 1e-5, False)      # one Llama-3-8B layer
eng = E.CrAMEngine.random(sp, dev, seed=1, std=0.02)
eng.no_tail_split = NO_TAIL
lw = eng.layers[0]
wil = eng._gate_up_interleaved(lw)
T = 1000
cos, sin = eng.rope_tables(T)
X = torch.randn(hi, 4096, device=dev).to(torch.bfloat16)
A = torch.randn(hi, 14336, device=dev).to(torch.bfloat16)
H = torch.randn(hi, 4096, device=dev).to(torch.bfloat16)


def layer(M):
    x, a, h = X[:M], A[:M], H[:M]
    ops.gemm_rope(x, lw.wqkv, sp.num_heads, sp.num_kv_heads, sp.head_dim, cos, sin, T, rows=M)
    eng._gemm_residual(x, lw.wo, h)
    ops.gemm(x, wil, ops.GEMM_SILU_MUL)
    eng._gemm_residual(a, lw.wd, h)


Ms = list(range(lo, hi + 1, step))
res = {M: [] for M in Ms}
for rnd in range(rounds):
    for M in Ms:
        layer(M)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            layer(M)
        e.record()
        torch.cuda.synchronize()
        res[M].append(s.elapsed_time(e) / 3)
    print(f"round {rnd} done", file=sys.stderr, flush=True)
tail = "without" if NO_TAIL else "with"
print(json.dumps({"note": "Median ms of one Llama-3-8B suffix layer's four projection GEMMs as the engine runs them "
                          f"(q/k/v + RoPE, o_proj + residual {tail} the tail split, gate/up + SiLU-mul, down + residual "
                          f"{tail} the tail split; bf16) per row count M on one MI355X (tools/gemm_rows_sweep.py "
                          f"{lo} {hi} {step} {rounds}{' no-tail' if NO_TAIL else ''}).  Used by engine.padded_rows.",
                  "shape": {"hidden": 4096, "intermediate": 14336, "qkv": 6144},
                  ("layer_gemm_ms_no_tail" if NO_TAIL else "layer_gemm_ms"):
                      {str(M): round(statistics.median(v), 4) for M, v in res.items()}}))
