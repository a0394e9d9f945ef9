"""Driver for rocprofv3 PMC passes on the sweep's dominant launch: gemm_w4_kernel with the SiLU-mul epilogue (gate/up,
~51 % of the sweep's GPU time) at the sweep shape M x 28,672 x 4,096 (tools/pmc_gemm.sh runs one counter set per
pass, restricted to gemm_w4_kernel dispatches).
    python tools/gemm_pmc.py [M] [iters]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import ops  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 29184
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
D, F = 4096, 14336
x = (torch.rand(M, D, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
wgu = ((torch.rand(2 * F, D, device=dev, generator=g) * 2 - 1) * D ** -0.5).to(torch.bfloat16)
wil = ops.interleave_gate_up(wgu, F)
for _ in range(iters):
    ops.gemm(x, wil, ops.GEMM_SILU_MUL)
torch.cuda.synchronize()
print("done")
