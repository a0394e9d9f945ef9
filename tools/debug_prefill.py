import torch, math, sys
sys.path.insert(0, '.')
from cram_amd import ops
from oracle import hook_ref
dev = torch.device('cuda:0')
torch.set_printoptions(precision=4, linewidth=200)
d = 128
for T in (2, 5, 17):
    # (a) q = 0 -> uniform attention over causal keys: out[i] = mean(V[:i+1])
    q = torch.zeros(1, 1, T, d, dtype=torch.bfloat16)
    k = torch.randn(1, 1, T, d).to(torch.bfloat16)
    v = torch.zeros(1, 1, T, d)
    for j in range(T):
        v[0, 0, j, :] = j + 1
    v = v.to(torch.bfloat16)
    out = ops.attn_prefill(q.to(dev), k.to(dev), v.to(dev), scale=d ** -0.5)
    torch.cuda.synchronize()
    print('T', T, 'uniform: got', out[0, :, 0, :4].float().cpu().tolist())
    print('   want', [(i + 2) / 2 for i in range(T)])
    # (b) random
    q = torch.randn(1, 1, T, d).to(torch.bfloat16); v = torch.randn(1, 1, T, d).to(torch.bfloat16)
    ref = hook_ref.biased_attention_ref(q, k, v, None, None, d ** -0.5)
    out = ops.attn_prefill(q.to(dev), k.to(dev), v.to(dev), scale=d ** -0.5)
    torch.cuda.synchronize()
    print('   random max err per row', (out.double().cpu() - ref).abs().amax(dim=(0, 2, 3)).tolist())
