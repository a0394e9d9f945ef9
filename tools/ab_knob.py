"""Same-process A/B of two prefill kernel selections (CRAM_KNOB_PREFILL_VARIANT values) on the IE sweep's shapes:
interleaved rounds, medians of 10-launch timings, outputs compared bit for bit.
  python tools/ab_knob.py [A=4] [B=5] [rounds=7]"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from cram_amd import _lib, ops  # noqa: E402

A = int(sys.argv[1]) if len(sys.argv) > 1 else 4
Bk = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
dev = torch.device("cuda:0")
d = 128
cases = []
for B, T, biased, p0 in [(33, 962, False, 0), (33, 937, False, 25), (33, 880, True, 25), (1, 962, True, 0),
                         (1, 8300, False, 0), (16, 8300, True, 0)]:
    g = torch.Generator(device=dev).manual_seed(B * T + p0)
    y = torch.randn(B, T + p0, 48 * d, device=dev, generator=g).to(torch.bfloat16)
    q = y[:, p0:, :32 * d].unflatten(-1, (32, d)).transpose(1, 2)
    k = y[..., 32 * d:40 * d].unflatten(-1, (8, d)).transpose(1, 2)
    v = y[..., 40 * d:].unflatten(-1, (8, d)).transpose(1, 2)
    bias = enable = None
    W = 0
    if biased:
        bias = torch.zeros(B, T + p0, device=dev)
        bias[:, 40:400] = -2.3
        bias[:, 500:700] = float("-inf")
        enable = torch.zeros(B, 32, dtype=torch.uint8, device=dev)
        enable[:, ::3] = 1
        W = T + p0
    fl, _ = ops.prefill_work(B, 32, 8, T, T + p0, d, p0)
    cases.append(((B, T, biased, p0), q, k, v, bias, enable, W, fl))


def call(q, k, v, bias, enable, W, out):
    return ops.attn_prefill(q, k, v, scale=d ** -0.5, bias=bias, enable=enable, W=W, out=out)


prev = _lib.get_knob(_lib.KNOB_PREFILL_VARIANT)
outs = {}
for knob in (A, Bk):
    _lib.set_knob(_lib.KNOB_PREFILL_VARIANT, knob)
    for name, q, k, v, bias, enable, W, _ in cases:
        o = torch.empty(q.shape[0], q.shape[2], 32, d, device=dev, dtype=torch.bfloat16)
        call(q, k, v, bias, enable, W, o)
        outs[(knob, name)] = o
torch.cuda.synchronize()
for name, *_ in cases:
    same = torch.equal(outs[(A, name)], outs[(Bk, name)])
    print(f"{name}: outputs {'bit-identical' if same else 'DIFFER max ' + str((outs[(A, name)].float() - outs[(Bk, name)].float()).abs().max().item())}", flush=True)
res = {(kn, c[0]): [] for kn in (A, Bk) for c in cases}
for _ in range(rounds):
    for kn in (A, Bk):
        _lib.set_knob(_lib.KNOB_PREFILL_VARIANT, kn)
        for name, q, k, v, bias, enable, W, _ in cases:
            o = outs[(kn, name)]
            for _ in range(2):
                call(q, k, v, bias, enable, W, o)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call(q, k, v, bias, enable, W, o)
            e1.record()
            torch.cuda.synchronize()
            res[(kn, name)].append(e0.elapsed_time(e1) / 10)
_lib.set_knob(_lib.KNOB_PREFILL_VARIANT, prev)
for name, *_, fl in cases:
    ta, tb = statistics.median(res[(A, name)]), statistics.median(res[(Bk, name)])
    print(f"{str(name):24s} knob {A}: {ta:.3f} ms ({fl / ta / 1e9:5.0f} TF/s, {fl / ta / 2.5e12:.3f})  knob {Bk}: "
          f"{tb:.3f} ms ({fl / tb / 1e9:5.0f} TF/s, {fl / tb / 2.5e12:.3f})  {Bk}/{A} speed {ta / tb:.3f}x", flush=True)
