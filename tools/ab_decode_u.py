"""Same-process A/B of the decode bodies at the decode leg's shape (B sequences of ragged length, Llama-3 GQA 4:1
by default, credibility bias on half the heads): the VALU kernel with U = 4 / 2 / 1 keys per lane group (knob
CRAM_KNOB_DECODE_U, matrix cores off) and the matrix-core kernel ("m", knob CRAM_KNOB_DECODE_MFMA).

    [AB_HEADS=Hq,Hkv,d] [AB_SPLITS=n] python tools/ab_decode_u.py [B] [S] [variant list, e.g. m,4,2,1]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cram_amd import _lib, ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
Hq, Hkv, d = (int(x) for x in os.environ.get("AB_HEADS", "32,8,128").split(","))
SPLITS = int(os.environ.get("AB_SPLITS", "1"))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
kc = torch.randn(B, Hkv, S, d, device=dev, generator=g).to(torch.bfloat16)
vc = torch.randn(B, Hkv, S, d, device=dev, generator=g).to(torch.bfloat16)
q = torch.randn(B, Hq, d, device=dev, generator=g).to(torch.bfloat16)
lens = torch.randint(int(S * 0.75), S - 16, (B,), device=dev, generator=g).to(torch.int32)
bias = torch.zeros(B, S, device=dev)
bias[:, 40:200] = -2.296875
enable = (torch.rand(B, Hq, device=dev, generator=g) < 0.5).to(torch.uint8)
kv_bytes = float(lens.sum()) * Hkv * d * 2 * 2
out = torch.empty_like(q)
ref = None
res = {}
for rnd in range(5):
    for u in (sys.argv[3].split(",") if len(sys.argv) > 3 else ("m", "4", "2", "1")):
        _lib.set_knob(_lib.KNOB_DECODE_MFMA, 1 if u == "m" else 0)
        _lib.set_knob(_lib.KNOB_DECODE_U, -1 if u == "m" else int(u))
        run = lambda: ops.attn_decode(q, kc, vc, scale=d ** -0.5, seq_lens=lens, bias=bias, enable=enable, W=S,
                                      out=out, num_splits=SPLITS)
        run()
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        assert (out.float() - ref.float()).abs().max().item() < 2e-2, u
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            run()
        e.record()
        torch.cuda.synchronize()
        res.setdefault(u, []).append(s.elapsed_time(e) / 20)
for u, v in res.items():
    ms = statistics.median(v)
    print(f"{'mfma' if u == 'm' else 'valu U=' + u}: {ms * 1e3:.1f} us, {kv_bytes / (ms * 1e-3) / 1e9:.0f} GB/s", flush=True)
