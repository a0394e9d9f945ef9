"""Driver for rocprofv3 PMC passes on the sweep's dominant launch: gemm_w4_kernel with the SiLU-mul epilogue (gate/up,
~51 % of the sweep's GPU time) at the sweep shape M x 28,672 x 4,096 (tools/pmc_gemm.sh runs one counter set per
pass, restricted to gemm_w4_kernel dispatches).
    python tools/gemm_pmc.py [M] [iters] [mode]
mode: silu (default: the 4-wave kernel's SiLU-mul epilogue), store (the 4-wave kernel, plain store), lt (hipBLASLt
F.linear of the same [gate; up] product: the library kernel's clock / MFMA-busy / traffic under the same counters)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import ops  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 29184
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
mode = sys.argv[3] if len(sys.argv) > 3 else "silu"
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
D, F = 4096, 14336
x = (torch.rand(M, D, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
wgu = ((torch.rand(2 * F, D, device=dev, generator=g) * 2 - 1) * D ** -0.5).to(torch.bfloat16)
wil = ops.interleave_gate_up(wgu, F)
torch.backends.cuda.preferred_blas_library("hipblaslt")
for _ in range(iters):
    if mode == "lt":
        torch.nn.functional.linear(x, wgu)
    elif mode == "store":
        ops.gemm(x, wil)
    else:
        ops.gemm(x, wil, ops.GEMM_SILU_MUL)
torch.cuda.synchronize()
print("done")
