"""CredibilityBias: the O(S) descriptor that replaces the hook's dense [1, H, T, S] mask.

The reference's forward-pre-hook (re_weighting.py:36-61) writes, for every
selected head h and every causal-allowed (i, j) with j < W,
      mask[0, h, i, j] = dtype(log_fp16(w_j))
where w is the fp16 weight vector (re_weighting.py:99,111), the log is taken on
the fp16 tensor (re_weighting.py:122,166) and the cast target is the hidden-state
dtype (re_weighting.py:56).  Because the allowed entries of the causal mask are
0, "replace" equals "add".  So the whole mask is described by

      bias[b, j]        = float(dtype(log_fp16(w_j)))   for j < W   (0 beyond W)
      enable[l, b, h]   = 1 if head h of layer l is selected

and the kernels add enable * bias to the fp32 scores inline.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, Optional, Sequence

import torch


def bias_from_weight(w16: torch.Tensor, model_dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """fp16 weights [B, W] -> fp32 bias [B, W] holding exactly the value the hook writes."""
    if w16.dtype != torch.float16:
        raise TypeError("credibility weights are fp16 in the reference (re_weighting.py:99)")
    return torch.log(w16.cpu()).to(model_dtype).float()


def head_enable(layers_to_heads: Dict, num_layers: int, num_heads: int) -> torch.Tensor:
    """{layer: [heads]} (keys may be str, as loaded from selected_heads.json) -> uint8 [L, Hq]."""
    en = torch.zeros((num_layers, num_heads), dtype=torch.uint8)
    for l, hs in layers_to_heads.items():
        l = int(l)
        if not 0 <= l < num_layers:
            raise ValueError(f"layer {l} out of range")
        for h in hs:
            if not 0 <= int(h) < num_heads:
                raise ValueError(f"head {h} out of range")
            en[l, int(h)] = 1
    return en


def all_heads(num_layers: int, num_heads: int) -> Dict[int, list]:
    """Empty layers_to_be_modified means every head of every layer (re_weighting.py:32-33)."""
    return {i: list(range(num_heads)) for i in range(num_layers)}


@dataclass
class CredibilityBias:
    """Device-resident descriptor for one batch of prompts.

    bias   : fp32 [B, S_cap]  (natural-log units, zero for j >= W_b)
    enable : uint8 [L, B, Hq]
    W      : max over the batch of the biased prefix length (keys >= W_b carry 0 anyway)
    """
    bias: torch.Tensor
    enable: torch.Tensor
    W: int

    @staticmethod
    def build(weights16: Sequence[torch.Tensor], layers_to_heads: Dict, num_layers: int, num_heads: int,
              device, model_dtype=torch.bfloat16, s_cap: Optional[int] = None,
              per_sample_heads: Optional[Iterable[Dict]] = None) -> "CredibilityBias":
        B = len(weights16)
        W = max(int(w.shape[-1]) for w in weights16)
        cap = max(W, s_cap or 0)
        bias = torch.zeros((B, cap), dtype=torch.float32)
        for b, w in enumerate(weights16):
            row = bias_from_weight(w.reshape(1, -1), model_dtype)[0]
            bias[b, :row.shape[0]] = row
        if per_sample_heads is None:
            en = head_enable(layers_to_heads, num_layers, num_heads)[:, None, :].expand(num_layers, B, num_heads)
        else:
            en = torch.stack([head_enable(h, num_layers, num_heads) for h in per_sample_heads], 1)
        return CredibilityBias(bias.to(device), en.contiguous().to(device), W)

    def layer_enable(self, layer: int) -> torch.Tensor:
        return self.enable[layer]
