"""Diagnose cram_gemm_rope against cram_gemm + cram_rope_inplace: which columns / rows differ, and whether the
raw projection (identity tables: cos 1, sin 0) already differs.
  python tools/gemm_rope_probe.py [K]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import ops  # noqa: E402

HQ, HKV, HD = 32, 8, 128


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(41 + K)
    M, T = 3072, 1000
    rows = 3000
    N = (HQ + 2 * HKV) * HD
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).to(dev)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) * K ** -0.5).to(torch.bfloat16).to(dev)
    a = ops.gemm(x, w)
    b = ops.gemm(x, w)
    print("gemm twice equal:", torch.equal(a, b), flush=True)
    one = torch.ones(T, HD, dtype=torch.bfloat16, device=dev)
    zero = torch.zeros(T, HD, dtype=torch.bfloat16, device=dev)
    r = ops.gemm_rope(x, w, HQ, HKV, HD, one, zero, T, rows=rows)
    d = (r[:rows] != a[:rows])
    print("identity-table rope vs gemm: differing elements", int(d.sum()), flush=True)
    if d.any():
        idx = d.nonzero()
        print(" rows", idx[:, 0].unique()[:20].tolist(), flush=True)
        print(" cols", idx[:, 1].unique()[:40].tolist(), flush=True)
        cols = idx[:, 1]
        print(" by head kind: q", int((cols < HQ * HD).sum()), "k", int(((cols >= HQ * HD) & (cols < (HQ + HKV) * HD)).sum()),
              "v", int((cols >= (HQ + HKV) * HD).sum()), flush=True)
        ref = x.float() @ w.float().t()
        i0 = idx[0]
        print(" first", i0.tolist(), "rope", r[i0[0], i0[1]].item(), "gemm", a[i0[0], i0[1]].item(),
              "fp32", ref[i0[0], i0[1]].item(), flush=True)


if __name__ == "__main__":
    main()
