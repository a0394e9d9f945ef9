import sys, torch
sys.path.insert(0, '.')
from cram_amd import ops
from cram_amd.engine import CrAMEngine, ModelSpec
dev = torch.device('cuda:0')
d, Hq, Hkv = 128, 32, 8
sp = ModelSpec(1, Hq * d, Hq, Hkv, d, 256, 100, 1e-5, False)
eng = CrAMEngine.random(sp, dev, seed=1)
B, T = 2, 131
N = (Hq + 2 * Hkv) * d
y = torch.randn(B, T, N, device=dev).to(torch.bfloat16)
cos, sin = eng.rope_tables(T)
x = y[..., :(Hq + Hkv) * d].unflatten(-1, (Hq + Hkv, d))
c, s = cos[None, :, None, :], sin[None, :, None, :]
rot = torch.cat((-x[..., d // 2:], x[..., :d // 2]), dim=-1)
t1 = x * c; t2 = rot * s
ref = t1 + t2
# emulate kernel formula in torch float
xf = x.float(); cf = c.float(); sf = s.float(); rf = rot.float()
emu = ((xf * cf).to(torch.bfloat16).float() + (rf * sf).to(torch.bfloat16).float()).to(torch.bfloat16)
print('emu==ref', torch.equal(emu, ref))
yy = y.clone()
ops.rope_inplace(yy, Hq + Hkv, d, cos, sin, T)
got = yy[..., :(Hq + Hkv) * d].unflatten(-1, (Hq + Hkv, d))
bad = got != ref
print('mismatch frac', bad.float().mean().item())
idx = bad.nonzero()
print(idx[:10].tolist())
for b_, t_, h_, i_ in idx[:5].tolist():
    print(got[b_, t_, h_, i_].item(), ref[b_, t_, h_, i_].item(), emu[b_, t_, h_, i_].item(), t1[b_,t_,h_,i_].item(), t2[b_,t_,h_,i_].item())
