"""Tiny random-weight Llama-3 / Qwen2 / Llama-2 / GPT-2 models with deterministic, documented weights.

No checkpoint is committed.  Every parameter tensor is drawn from numpy's PCG64
stream seeded with SeedSequence([seed, crc32(parameter name)]) (stable across
numpy versions and machines), scaled by a per-kind std, then rounded to the
kind's dtype (bf16; fp16 for the Llama-2 stand-in, whose checkpoints the
reference loads as fp16 through torch_dtype="auto").
The golden vectors in tests/golden/ were produced by the reference running on
exactly these weights, so any machine can rebuild the same model.
"""
from __future__ import annotations

import os
import zlib

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOK_DIR = {"llama3": os.path.join(REPO, "data", "tok_llama3"), "qwen2": os.path.join(REPO, "data", "tok_qwen"),
           "gpt2": os.path.join(REPO, "data", "tok_llama3"), "llama2": os.path.join(REPO, "data", "tok_llama3")}
# names select the reference's chat branch; "gpt2-tiny" and "Llama-2-tiny" match neither, i.e. the
# raw-template branch (the reference's default model, Llama-2-13b-chat-hf, takes that branch too)
DIR_NAME = {"llama3": "Llama-3-tiny", "qwen2": "Qwen2-tiny", "gpt2": "gpt2-tiny", "llama2": "Llama-2-tiny",
            "qwen2_7b": "Qwen2-7B-heads-2layer", "qwen2_gqa7": "Qwen2-GQA7-tiny"}
TOK_DIR["qwen2_7b"] = TOK_DIR["qwen2"]
TOK_DIR["qwen2_gqa7"] = TOK_DIR["qwen2"]
DTYPE = {"llama2": torch.float16}

SPECS = {
    "llama3": dict(hidden_size=256, intermediate_size=512, num_hidden_layers=4, num_attention_heads=4,
                   num_key_value_heads=2, head_dim=128, rope_theta=500000.0, rms_norm_eps=1e-5,
                   max_position_embeddings=4096, tie_word_embeddings=False),
    "qwen2": dict(hidden_size=256, intermediate_size=512, num_hidden_layers=3, num_attention_heads=2,
                  num_key_value_heads=1, rope_theta=1000000.0, rms_norm_eps=1e-6,
                  max_position_embeddings=4096, tie_word_embeddings=False),
    # GPT-2 architecture (config 1's family): MHA, head_dim 64, learned positions, LayerNorm, GELU
    "gpt2": dict(n_embd=256, n_inner=512, n_layer=3, n_head=4, n_positions=4096),
    # Llama-2-13b's shape family: MHA (kv heads == heads), head_dim 128, rope_theta 1e4, fp16
    "llama2": dict(hidden_size=256, intermediate_size=512, num_hidden_layers=3, num_attention_heads=4,
                   num_key_value_heads=4, head_dim=128, rope_theta=10000.0, rms_norm_eps=1e-5,
                   max_position_embeddings=4096, tie_word_embeddings=False),
    # config 4's layout at full width (Qwen2-7B: D 3584, 28 q / 4 kv heads of 128, FFN 18944, q/k/v bias,
    # rope 1e6), two layers: the GQA-7 kernels and the decode projections at their real shapes
    "qwen2_7b": dict(hidden_size=3584, intermediate_size=18944, num_hidden_layers=2, num_attention_heads=28,
                     num_key_value_heads=4, rope_theta=1000000.0, rms_norm_eps=1e-6,
                     max_position_embeddings=4096, tie_word_embeddings=False),
    # Qwen2-7B's head grouping (7 q-heads per kv head, head_dim 128, q/k/v bias, rope 1e6) at 4 layers x 14 heads
    # (2 kv heads): 56 IE values per question (the 3 x 2 "qwen2" kind has 6), the GQA-7 attention kernels and every
    # fused GEMM epilogue (widths as Qwen2-7B's: hidden a multiple of 256, an even q/k/v head count) on the
    # reference-pinned path
    "qwen2_gqa7": dict(hidden_size=1792, intermediate_size=2048, num_hidden_layers=4, num_attention_heads=14,
                       num_key_value_heads=2, rope_theta=1000000.0, rms_norm_eps=1e-6,
                       max_position_embeddings=4096, tie_word_embeddings=False),
}
# linear-weight std per kind (fan-in 256 for the tiny kinds; wider kinds keep the activations O(1): std ~ 1.3/sqrt(fan-in))
LIN_STD_KIND = {"qwen2_7b": 0.02, "qwen2_gqa7": 0.03}
SEED = 20250404
LIN_STD = 0.08


def dtype(kind: str) -> torch.dtype:
    return DTYPE.get(kind, torch.bfloat16)


def _draw(name: str, shape, std: float, mean: float = 0.0, seed: int = SEED, dt=torch.bfloat16) -> torch.Tensor:
    rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, zlib.crc32(name.encode())])))
    a = rng.standard_normal(size=shape, dtype=np.float32) * np.float32(std) + np.float32(mean)
    return torch.from_numpy(a).to(dt)


def tokenizer(kind: str):
    from transformers import AutoTokenizer
    return AutoTokenizer.from_pretrained(TOK_DIR[kind])


def config(kind: str):
    from transformers import GPT2Config, LlamaConfig, Qwen2Config
    tok = tokenizer(kind)
    spec = dict(SPECS[kind])
    if kind == "gpt2":
        cfg = GPT2Config(vocab_size=len(tok), bos_token_id=tok.bos_token_id, eos_token_id=tok.eos_token_id, **spec)
    elif kind in ("llama3", "llama2"):
        cfg = LlamaConfig(vocab_size=len(tok), bos_token_id=tok.bos_token_id, eos_token_id=tok.eos_token_id,
                          **spec)
    else:
        cfg = Qwen2Config(vocab_size=len(tok), eos_token_id=tok.eos_token_id, **spec)
    cfg.torch_dtype = dtype(kind)
    return cfg


def build_model(kind: str, attn_implementation: str = "sdpa"):
    """The tiny model on CPU in its dtype (bf16, fp16 for llama2) with the deterministic weights."""
    from transformers import AutoModelForCausalLM
    from functools import partial
    cfg = config(kind)
    model = AutoModelForCausalLM.from_config(cfg, attn_implementation=attn_implementation, dtype=dtype(kind))
    draw = partial(_draw, dt=dtype(kind))
    sd = {}
    for name, p in model.state_dict().items():
        if name.endswith("norm.weight") or "layernorm" in name or (".ln_" in name and name.endswith("weight")):
            sd[name] = draw(name, tuple(p.shape), 0.1, 1.0)
        elif name.endswith(".attn.bias") or name.endswith(".masked_bias"):   # GPT-2 causal buffers, not weights
            sd[name] = p
        elif name.endswith("wte.weight") or name.endswith("wpe.weight"):        # GPT-2: tied lm_head
            sd[name] = draw(name, tuple(p.shape), 0.3 if name.endswith("wte.weight") else 0.1)
        elif name.endswith("embed_tokens.weight"):
            sd[name] = draw(name, tuple(p.shape), 1.0)
        elif name.endswith(".bias"):
            sd[name] = draw(name, tuple(p.shape), 0.05)
        else:
            sd[name] = draw(name, tuple(p.shape), LIN_STD_KIND.get(kind, LIN_STD))
    model.load_state_dict(sd)
    model.eval()
    return model


def save_model(kind: str, root: str, fp32: bool = False) -> str:
    """Write the tiny model + tokenizer as a local HF directory (name selects the chat branch).

    fp32=True stores the same (bf16- / fp16-valued) weights widened to float32: the
    float32 reference run of that model is the IE ground truth of the tests.
    """
    path = os.path.join(root, DIR_NAME[kind] + ("-f32" if fp32 else ""))
    if not os.path.exists(os.path.join(path, "config.json")):
        os.makedirs(path, exist_ok=True)
        m = build_model(kind)
        if fp32:
            m = m.float()
            m.config.torch_dtype = torch.float32
        m.save_pretrained(path)
        tokenizer(kind).save_pretrained(path)
    return path
