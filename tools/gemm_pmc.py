"""Driver for rocprofv3 PMC passes on the gate/up GEMM: cram_gemm (store and fused SiLU-mul) and hipBLASLt at the
sweep shape, a few launches each (tools/gemm_pmc.sh runs one counter set per pass)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import ops  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 29184
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
torch.backends.cuda.preferred_blas_library("hipblaslt")
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
D, F = 4096, 14336
x = (torch.rand(M, D, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
wgu = ((torch.rand(2 * F, D, device=dev, generator=g) * 2 - 1) * D ** -0.5).to(torch.bfloat16)
wil = ops.interleave_gate_up(wgu, F)
for _ in range(iters):
    torch.nn.functional.linear(x, wgu)
    ops.gemm(x, wgu)
    ops.gemm(x, wil, ops.GEMM_SILU_MUL)
torch.cuda.synchronize()
print("done")
