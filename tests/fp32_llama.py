"""Plain-PyTorch float32 reference of the hooked Llama/Qwen2 forward, for parity tests at BASELINE sizes.

Test infrastructure only.  It restates, in float32 and with the dense additive mask the reference hook builds
(re_weighting.py:36-61: causal mask, the selected heads' causal-allowed entries replaced by log w_j for j < W),
the decoder stack that transformers runs under the hook (RMSNorm, RoPE, GQA SDPA, SwiGLU MLP), on the weights of a
CrAMEngine upcast to float32.  It is the ground truth the bf16 paths are measured against: the IE of one unit
(layer l, head h) is re_weighting.py:152-175's  sum_k logit(a_k) unhooked - sum_k logit(a_k) hooked, read at the
positions of the answer tokens themselves (:160,170).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class Fp32Llama:
    def __init__(self, eng):
        sp = eng.spec
        self.sp = sp
        f = lambda t: None if t is None else t.float()
        self.layers = [dict(ln1=f(lw.ln1), wqkv=f(lw.wqkv), bqkv=f(lw.bqkv), wo=f(lw.wo), ln2=f(lw.ln2),
                            wgu=f(lw.wgu), wd=f(lw.wd)) for lw in eng.layers]
        self.embed = eng.embed
        self.norm = f(eng.norm)
        self.lm_head = eng.lm_head
        self.inv_freq = eng.inv_freq.float()
        self.attn_scaling = eng.attn_scaling

    def rms(self, x, w):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + self.sp.eps) * w

    def rope(self, T, dev):
        fr = torch.arange(T, device=dev, dtype=torch.float32)[:, None] * self.inv_freq[None, :]
        emb = torch.cat((fr, fr), -1)
        return emb.cos() * self.attn_scaling, emb.sin() * self.attn_scaling

    @staticmethod
    def rot(x, cos, sin):
        d = x.shape[-1] // 2
        return x * cos + torch.cat((-x[..., d:], x[..., :d]), -1) * sin

    def layer(self, h, l, cos, sin, mask):
        """h [T, D] fp32; mask [Hq, T, T] additive fp32 (causal + hook bias)."""
        sp, w = self.sp, self.layers[l]
        T = h.shape[0]
        x = self.rms(h, w["ln1"])
        y = x @ w["wqkv"].t()
        if w["bqkv"] is not None:
            y = y + w["bqkv"]
        q = y[:, :sp.q_size].view(T, sp.num_heads, sp.head_dim).transpose(0, 1)
        k = y[:, sp.q_size:sp.q_size + sp.kv_size].view(T, sp.num_kv_heads, sp.head_dim).transpose(0, 1)
        v = y[:, sp.q_size + sp.kv_size:].view(T, sp.num_kv_heads, sp.head_dim).transpose(0, 1)
        q, k = self.rot(q, cos, sin), self.rot(k, cos, sin)
        g = sp.num_heads // sp.num_kv_heads
        k, v = k.repeat_interleave(g, 0), v.repeat_interleave(g, 0)
        a = F.scaled_dot_product_attention(q[None], k[None], v[None], attn_mask=mask[None])[0]
        h = h + a.transpose(0, 1).reshape(T, sp.q_size) @ w["wo"].t()
        x2 = self.rms(h, w["ln2"])
        gu = x2 @ w["wgu"].t()
        act = F.silu(gu[:, :sp.intermediate]) * gu[:, sp.intermediate:]
        return h + act @ w["wd"].t()

    def causal(self, T, dev):
        return torch.full((T, T), float("-inf"), device=dev).triu(1)

    @torch.no_grad()
    def baseline(self, ids):
        """Un-hooked forward: per-layer inputs [L][T, D] and the final hidden states [T, D]."""
        T = ids.numel()
        dev = self.norm.device
        cos, sin = self.rope(T, dev)
        mask = self.causal(T, dev).expand(self.sp.num_heads, T, T)
        h = self.embed[ids.view(-1)].float()
        hs = []
        for l in range(self.sp.num_layers):
            hs.append(h)
            h = self.layer(h, l, cos, sin, mask)
        return hs, self.rms(h, self.norm)

    def answer_sum(self, hfinal, ans):
        """sum_k <h[-n+k], lm_head[a_k]> in float32 (re_weighting.py:160)."""
        n = ans.numel()
        return (hfinal[-n:] * self.lm_head[ans.long()].float()).sum()

    @torch.no_grad()
    def ie_units(self, ids, bias, ans, units):
        """IE of each (layer, head) unit: one hooked forward from that layer's cached input.

        bias: fp32 [W] per-key hook value (log w_j, -inf for weight 0); W <= T."""
        T = ids.numel()
        dev = self.norm.device
        cos, sin = self.rope(T, dev)
        hs, hf = self.baseline(ids)
        ori = self.answer_sum(hf, ans)
        causal = self.causal(T, dev)
        hooked = causal.clone()
        W = bias.numel()
        allowed = causal[:, :W] == 0
        hooked[:, :W] = torch.where(allowed, bias[None, :].expand(T, W), causal[:, :W])   # replace, :57-59
        out = []
        for l, hh in units:
            mask = causal.repeat(self.sp.num_heads, 1, 1)
            mask[hh] = hooked
            h = hs[l]
            for l2 in range(l, self.sp.num_layers):
                h = self.layer(h, l2, cos, sin, mask if l2 == l else causal.expand(self.sp.num_heads, T, T))
            out.append(float(ori - self.answer_sum(self.rms(h, self.norm), ans)))
        return out

    @torch.no_grad()
    def ie_grid(self, ids, bias, ans, layers=None):
        """IE [len(layers), H] float64 of every (layer, head) unit, computed per layer as a batch of H hooked
        variants (variant h: head h of layer l re-weighted; layers above l plain causal).  Mathematically the
        same units as ie_units (one hooked forward per unit); only the fp32 GEMM shapes differ."""
        sp = self.sp
        T = ids.numel()
        H = sp.num_heads
        dev = self.norm.device
        cos, sin = self.rope(T, dev)
        hs, hf = self.baseline(ids)
        ori = self.answer_sum(hf, ans)
        causal = self.causal(T, dev)
        hooked = causal.clone()
        W = bias.numel()
        allowed = causal[:, :W] == 0
        hooked[:, :W] = torch.where(allowed, bias[None, :].expand(T, W), causal[:, :W])   # replace, :57-59
        n = ans.numel()
        w_ans = self.lm_head[ans.long()].float()
        layers = range(sp.num_layers) if layers is None else layers
        out = torch.empty((len(layers), H), dtype=torch.float64)
        for i, l in enumerate(layers):
            mask = causal.repeat(H, H, 1, 1)                          # [variant, head, T, T]
            idx = torch.arange(H, device=dev)
            mask[idx, idx] = hooked
            h = hs[l].expand(H, T, sp.hidden).contiguous()
            for l2 in range(l, sp.num_layers):
                h = self.layer_batch(h, l2, cos, sin, mask if l2 == l else None)
            hn = self.rms(h[:, -n:], self.norm)                       # [H, n, D]
            cur = (hn * w_ans[None]).sum((1, 2))
            out[i] = (ori - cur).double().cpu()
        return out

    def layer_batch(self, h, l, cos, sin, mask):
        """layer() over a batch [B, T, D]; mask [B, Hq, T, T] additive, or None for plain causal."""
        sp, w = self.sp, self.layers[l]
        B, T, _ = h.shape
        x = self.rms(h, w["ln1"])
        y = x @ w["wqkv"].t()
        if w["bqkv"] is not None:
            y = y + w["bqkv"]
        q = y[..., :sp.q_size].view(B, T, sp.num_heads, sp.head_dim).transpose(1, 2)
        k = y[..., sp.q_size:sp.q_size + sp.kv_size].view(B, T, sp.num_kv_heads, sp.head_dim).transpose(1, 2)
        v = y[..., sp.q_size + sp.kv_size:].view(B, T, sp.num_kv_heads, sp.head_dim).transpose(1, 2)
        q, k = self.rot(q, cos, sin), self.rot(k, cos, sin)
        g = sp.num_heads // sp.num_kv_heads
        k, v = k.repeat_interleave(g, 1), v.repeat_interleave(g, 1)
        if mask is None:
            a = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        else:
            a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
        h = h + a.transpose(1, 2).reshape(B, T, sp.q_size) @ w["wo"].t()
        x2 = self.rms(h, w["ln2"])
        gu = x2 @ w["wgu"].t()
        act = F.silu(gu[..., :sp.intermediate]) * gu[..., sp.intermediate:]
        return h + act @ w["wd"].t()
