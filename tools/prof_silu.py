"""Live HBM rate of cram_silu_mul at the IE sweep's MLP shape (M rows x F=14336, bf16).

Algorithmic bytes per launch: read gate+up (2*F*2 B/row) + write y (F*2 B/row).
Prints GB/s for the HIP kernel and, beside it, torch's silu(g)*u (two kernels) as a yardstick.
Run on the GPU box: python tools/prof_silu.py
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from cram_amd import ops  # noqa: E402


def rate(fn, nbytes, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    return ms, nbytes / ms / 1e6


def main():
    F = 14336
    for M in (4096, 28672):
        gu = torch.randn(M, 2 * F, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
        nbytes = M * F * 2 * 3
        ms, gbs = rate(lambda: ops.silu_mul(gu, F, out=y), nbytes)
        ref = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
        assert torch.equal(ops.silu_mul(gu, F, out=y), ref), "silu_mul differs from torch"
        tms, tgbs = rate(lambda: torch.nn.functional.silu(gu[:, :F]) * gu[:, F:], nbytes)
        print(f"M={M} F={F}: cram_silu_mul {ms:.3f} ms {gbs:.0f} GB/s | torch silu*mul {tms:.3f} ms {tgbs:.0f} GB/s",
              flush=True)


if __name__ == "__main__":
    main()
