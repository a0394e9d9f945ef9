"""fp16 models on the HIP path: the reference's default model family (Llama-2-13b-chat-hf) is an fp16
checkpoint, and the reference loads it with torch_dtype="auto" (re_weighting.py:22), so its hooked SDPA,
RMSNorm, RoPE and MLP run in fp16 and the hook writes fp16(log_fp16(w)) into the mask.

Kernels: the fp16 instantiations against the oracle (float64 softmax over the hook's fp16 mask) with the
bf16 suite's tolerances, and the elementwise kernels against transformers' fp16 op sequences.
End to end: the fp16 MHA Llama-2 stand-in (tests/tiny_models.py "llama2") against the vectors the
reference produced on it (tests/golden/llama2_*.json.gz, gen_golden.py llama2) with the same noise-floor
bars as the bf16 families.
"""
import gzip
import json
import os

import numpy as np
import pytest
import torch

from oracle import hook_ref
from tests import parity
from tests import tiny_models as tm
from tests.test_engine_cpu import ie_tolerance_check
from tests.test_kernels_gpu import _check

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
F16 = torch.float16


def _load(name):
    with gzip.open(os.path.join(GOLD, name), "rt", encoding="utf-8") as f:
        return json.load(f)


def _bias16(B, Hq, W, gen):
    w = torch.ones((B, W), dtype=torch.float16)
    for (a, b, sc) in ((3, 40, 0.1), (41, 90, 0.0), (91, 150, 1.0), (151, 200, 0.5)):
        if a < W:
            w[:, a:min(b, W - 1) + 1] = sc
    lw = hook_ref.log_weight(w)
    bias = lw.to(F16).float()                      # the value the hook writes into an fp16 mask
    heads = [sorted(torch.randperm(Hq, generator=gen)[: max(1, Hq // 2)].tolist()) for _ in range(B)]
    enable = torch.zeros((B, Hq), dtype=torch.uint8)
    for b, hs in enumerate(heads):
        enable[b, hs] = 1
    return lw, bias, enable, heads


@pytest.mark.parametrize("B,Hq,Hkv,T,d", [(1, 40, 40, 300, 128), (2, 8, 2, 200, 128), (1, 4, 4, 129, 64),
                                          (1, 4, 1, 1, 128)])
@pytest.mark.parametrize("biased", [False, True])
def test_prefill_fp16(gpu_device, prefill_variant, B, Hq, Hkv, T, d, biased):
    from cram_amd import ops
    gen = torch.Generator().manual_seed(17 * T + Hq + biased)
    q = torch.randn(B, T, Hq, d, generator=gen).to(F16).transpose(1, 2)
    k = torch.randn(B, Hkv, T, d, generator=gen).to(F16)
    v = torch.randn(B, Hkv, T, d, generator=gen).to(F16)
    W = max(1, T - 3)
    lw, bias, enable, heads = _bias16(B, Hq, W, gen) if biased else (None, None, None, None)
    ref = hook_ref.biased_attention_ref(q, k, v, lw, heads, d ** -0.5, model_dtype=F16)
    dev = gpu_device
    out = ops.attn_prefill(q.to(dev), k.to(dev), v.to(dev), scale=d ** -0.5,
                           bias=None if bias is None else bias.to(dev),
                           enable=None if enable is None else enable.to(dev), W=W if biased else 0)
    torch.cuda.synchronize()
    assert out.dtype == F16
    _check(out, ref)


def test_prefill_fp16_zero_bias_is_no_bias(gpu_device, prefill_variant):
    """fp16 instantiation keeps the bf16 kernel's property: a zero bias is bit-identical to no bias."""
    from cram_amd import ops
    dev = gpu_device
    gen = torch.Generator(device=dev).manual_seed(5)
    B, Hq, Hkv, T, d = 2, 40, 40, 700, 128
    q = torch.randn(B, Hq, T, d, device=dev, generator=gen).to(F16)
    k = torch.randn(B, Hkv, T, d, device=dev, generator=gen).to(F16)
    v = torch.randn(B, Hkv, T, d, device=dev, generator=gen).to(F16)
    plain = ops.attn_prefill(q, k, v, scale=d ** -0.5)
    zero = ops.attn_prefill(q, k, v, scale=d ** -0.5, bias=torch.zeros((B, T), device=dev),
                            enable=torch.ones((B, Hq), dtype=torch.uint8, device=dev), W=T)
    assert torch.equal(plain, zero)


@pytest.mark.parametrize("B,Hq,Hkv,S,splits", [(2, 40, 40, 700, 1), (3, 40, 40, 1500, 4), (2, 8, 2, 333, 2)])
def test_decode_fp16(gpu_device, decode_variant, B, Hq, Hkv, S, splits):
    from cram_amd import ops
    d = 128
    gen = torch.Generator().manual_seed(S + splits)
    q = torch.randn(B, Hq, d, generator=gen).to(F16)
    k = torch.randn(B, Hkv, S + 3, d, generator=gen).to(F16)
    v = torch.randn(B, Hkv, S + 3, d, generator=gen).to(F16)
    lens = [max(1, S - 11 * b) for b in range(B)]
    W = S - 2
    lw, bias, enable, heads = _bias16(B, Hq, W, gen)
    ref = torch.cat([hook_ref.biased_attention_ref(q[b:b + 1, :, None], k[b:b + 1, :, :lens[b]],
                                                   v[b:b + 1, :, :lens[b]], lw[b:b + 1, :min(W, lens[b])], [heads[b]],
                                                   d ** -0.5, model_dtype=F16)[:, 0] for b in range(B)], 0)
    dev = gpu_device
    out = ops.attn_decode(q.to(dev), k.to(dev), v.to(dev), scale=d ** -0.5,
                          seq_lens=torch.tensor(lens, dtype=torch.int32, device=dev), bias=bias.to(dev),
                          enable=enable.to(dev), W=W, num_splits=splits)
    torch.cuda.synchronize()
    assert out.dtype == F16
    _check(out, ref)


def test_varlen_fp16(gpu_device, prefill_variant):
    from cram_amd import ops
    lens, Hq, Hkv, d = [17, 300, 1, 129], 8, 8, 128
    gen = torch.Generator().manual_seed(99)
    total = sum(lens)
    y = torch.randn(total, (Hq + 2 * Hkv) * d, generator=gen).to(F16)
    q = y[:, :Hq * d].view(total, Hq, d)
    k = y[:, Hq * d:(Hq + Hkv) * d].view(total, Hkv, d)
    v = y[:, (Hq + Hkv) * d:].view(total, Hkv, d)
    W = max(lens)
    lw, bias, enable, heads = _bias16(len(lens), Hq, W, gen)
    cu = np.concatenate([[0], np.cumsum(lens)]).tolist()
    ref = torch.cat([hook_ref.biased_attention_ref(q[a:e].transpose(0, 1)[None], k[a:e].transpose(0, 1)[None],
                                                   v[a:e].transpose(0, 1)[None], lw[b:b + 1, :e - a], [heads[b]],
                                                   d ** -0.5, model_dtype=F16)[0]
                     for b, (a, e) in enumerate(zip(cu[:-1], cu[1:]))], 0)
    dev = gpu_device
    yd = y.to(dev)
    out = ops.attn_prefill_varlen(yd[:, :Hq * d].view(total, Hq, d), yd[:, Hq * d:(Hq + Hkv) * d].view(total, Hkv, d),
                                  yd[:, (Hq + Hkv) * d:].view(total, Hkv, d),
                                  torch.tensor(cu, dtype=torch.int32, device=dev), max(lens), scale=d ** -0.5,
                                  bias=bias.to(dev), enable=enable.to(dev), W=W)
    torch.cuda.synchronize()
    _check(out, ref)


def test_answer_logits_fp16(gpu_device):
    from cram_amd import ops
    gen = torch.Generator().manual_seed(4)
    n, D, V = 29, 5120, 700
    h = torch.randn(n, D, generator=gen).to(F16)
    w = (torch.randn(V, D, generator=gen) * 0.02).to(F16)
    ids = torch.randint(0, V, (n,), generator=gen, dtype=torch.int32)
    ref = (h.double() * w[ids.long()].double()).sum(-1)
    dev = gpu_device
    out = ops.answer_logits(h.to(dev), w.to(dev), ids.to(dev))
    assert torch.allclose(out.double().cpu(), ref, atol=1e-3, rtol=1e-4)
    out16 = ops.answer_logits(h.to(dev), w.to(dev), ids.to(dev), round_logits=True)
    assert torch.equal(out16.cpu(), out.cpu().to(F16).float())
    with pytest.raises(TypeError):
        ops.answer_logits(h.to(dev), w.to(dev).to(torch.bfloat16), ids.to(dev))


def _ulp16(a, b):
    ai, bi = a.view(torch.int16).to(torch.int32), b.view(torch.int16).to(torch.int32)
    ai = torch.where(ai < 0, -(ai & 0x7FFF), ai)
    bi = torch.where(bi < 0, -(bi & 0x7FFF), bi)
    return (ai - bi).abs()


@pytest.mark.parametrize("D", [256, 5120])
def test_rmsnorm_fp16(gpu_device, D):
    from cram_amd import ops
    dev = gpu_device
    g = torch.Generator(device=dev).manual_seed(D)
    x = torch.randn(3, 77, D, device=dev, generator=g).to(F16)
    r = torch.randn(3, 77, D, device=dev, generator=g).to(F16)
    w = (1 + 0.1 * torch.randn(D, device=dev, generator=g)).to(F16)
    h = r + x
    hf = h.float()
    ref = w * (hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5)).to(F16)
    h_got, got = ops.rmsnorm(x, w, 1e-5, residual=r)
    assert torch.equal(h_got, h)
    ud = _ulp16(got, ref)
    # the fp32 mean differs from torch's in reduction order: an intermediate fp16 rounding can move by 1 ulp,
    # which w (up to ~1.3) can turn into 2 output ulps
    assert ud.max() <= 2 and (ud == 0).float().mean() > 0.995, (ud.max().item(), (ud == 0).float().mean().item())


def test_rope_fp16_bit_exact(gpu_device):
    from cram_amd import ops
    from cram_amd.engine import CrAMEngine, ModelSpec
    dev = gpu_device
    Hq = Hkv = 40
    d = 128
    sp = ModelSpec(1, Hq * d, Hq, Hkv, d, 256, 100, 1e-5, False)
    eng = CrAMEngine.random(sp, dev, seed=1, rope_theta=10000.0, dtype=F16)
    B, T = 2, 131
    y = torch.randn(B, T, (Hq + 2 * Hkv) * d, device=dev).to(F16)
    cos, sin = eng.rope_tables(T)
    assert cos.dtype == F16
    x = y[..., :(Hq + Hkv) * d].unflatten(-1, (Hq + Hkv, d))
    rot = torch.cat((-x[..., d // 2:], x[..., :d // 2]), dim=-1)
    ref = (x * cos[None, :, None, :]) + (rot * sin[None, :, None, :])
    ops.rope_inplace(y, Hq + Hkv, d, cos, sin, T)
    assert torch.equal(y[..., :(Hq + Hkv) * d].unflatten(-1, (Hq + Hkv, d)), ref)


def test_silu_mul_fp16(gpu_device):
    from cram_amd import ops
    F = 13824                                     # Llama-2-13b intermediate size
    gu = (2 * torch.randn(3, 50, 2 * F, device=gpu_device)).to(F16)
    ref = torch.nn.functional.silu(gu[..., :F]) * gu[..., F:]
    ud = _ulp16(ops.silu_mul(gu, F), ref)
    assert ud.max() <= 1 and (ud == 0).float().mean() > 0.995, (ud.max().item(), (ud == 0).float().mean().item())


# ---------------------------------------------------------------------------------------------- end to end
@pytest.fixture(scope="module")
def nq():
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def path(tmp_path_factory):
    return tm.save_model("llama2", str(tmp_path_factory.mktemp("llama2")))


def test_llama2_cal_logits_matches_reference(path, nq, gpu_device):
    from cram_amd.re_weighting import Find_Best_Heads
    obj = Find_Best_Heads(model_name=path)
    assert obj.model.dtype == F16 and obj.engine.dtype == F16
    gold = [x for x in _load("llama2_ie.json.gz") if x["variant"] == "fp32"]
    truth = {x["idx"]: x["ie"] for x in _load("llama2_ie_f32.json.gz")}
    agg = parity.Aggregate()
    for g in gold:
        rec = nq[g["idx"]]
        ie = obj.cal_logits(question=rec["question"], paras=rec["ori_fake"] + rec["reranked_dense_ctxs"],
                            scores=[0, 1, 1, 1, 1], wrong_answer=rec["wrong_answer"])
        ie_tolerance_check(ie, g["ie"], truth[g["idx"]], agg)
    agg.check()


@pytest.mark.parametrize("case", [0, 1])
def test_llama2_generate_matches_reference(path, nq, gpu_device, case):
    from cram_amd import attention as A
    from cram_amd.re_weighting import Re_Weighting_Strategy
    heads = [{0: [1], 2: [0, 3]}, {}][case]
    rows = [g for g in _load("llama2_generate.json.gz") if g["heads"] == {str(k): v for k, v in heads.items()}]
    obj = Re_Weighting_Strategy(model_name=path, layers_to_be_modified=dict(heads), bad_words_ids=[])
    for g in rows[:2]:
        rec = nq[g["idx"]]
        paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
        enc, w = obj.decode_with_special_attention(question=rec["question"], paras=paras, scores=[0.1, 1, 1, 1, 1])
        T = enc["input_ids"].shape[1]
        with A.reweighting(obj.model, obj._bias(w, obj.layers_to_be_modified)), torch.no_grad():
            out = obj.model.generate(**enc, **obj._generate_kwargs(), output_scores=True, return_dict_in_generate=True)
            last = obj.model(**enc).logits[0, -1].float().cpu()
        d = (last - torch.tensor(g["last_logits"])).abs()
        assert d.max() < 0.15 and d.mean() < 0.03, (d.max().item(), d.mean().item())
        ids, ref = out.sequences[0].tolist(), g["ids"]
        gaps = [(s[0].float().topk(2).values[0] - s[0].float().topk(2).values[1]).item() for s in out.scores]
        assert ids[:T] == ref[:T]
        for t in range(T, min(len(ids), len(ref))):
            if ids[t] != ref[t]:
                assert min(gaps[:t - T + 1]) < 0.05, (t - T, gaps[t - T])
                break
        else:
            assert len(ids) == len(ref)
            prompt, output = obj.run_RAG_with_attention_weighting(question=rec["question"], paras=paras,
                                                                  scores=[0.1, 1, 1, 1, 1])
            assert prompt == g["prompt"] and output == g["output"]


def test_llama2_logprobs_match_reference_hook(path, nq, gpu_device):
    from cram_amd.re_weighting import Re_Weighting_Strategy
    rows = _load("llama2_logprobs.json.gz")
    truth = {(r["idx"], r["scores"], r["heads"]): np.array(r["logprobs"]) for r in rows if r["fp32"]}
    objs = {}
    agg = parity.Aggregate()
    for r in rows:
        if r["fp32"]:
            continue
        if r["heads"] not in objs:
            objs[r["heads"]] = Re_Weighting_Strategy(model_name=path, layers_to_be_modified=r["layers_to_heads"])
        rec = nq[r["idx"]]
        scores = [0.1, 1, 1, 1, 1] if r["scores"] == "ideal" else [0, 1, 1, 1, 1]
        lp = objs[r["heads"]].answer_logprobs(question=rec["question"],
                                              paras=rec["ori_fake"] + rec["reranked_dense_ctxs"], scores=scores,
                                              answer=rec["wrong_answer"])
        t = truth[(r["idx"], r["scores"], r["heads"])]
        ref_err = np.abs(np.array(r["logprobs"]) - t).max()
        err = np.abs(lp.cpu().numpy() - t)
        agg.add("logprob_max", err.max(), ref_err, kind="llama2", idx=r["idx"], scores=r["scores"],
                heads=r["heads"])
    agg.check()


def test_llama2_engine_batched_decode(path, nq, gpu_device):
    """fp16 engine decode (packed varlen prefill + hipGraph step) == the transformers drop-in decode."""
    from cram_amd import attention as A
    from cram_amd.re_weighting import Re_Weighting_Strategy
    heads = {0: [1], 2: [0, 3]}
    obj = Re_Weighting_Strategy(model_name=path, layers_to_be_modified=heads, bad_words_ids=[])
    qs = [nq[i] for i in range(3)]
    args = ([q["question"] for q in qs], [q["ori_fake"] + q["reranked_dense_ctxs"] for q in qs],
            [[0.1, 1, 1, 1, 1]] * 3)
    graph = obj.run_RAG_batch(*args, max_new_tokens=16, use_graph=True)
    eager = obj.run_RAG_batch(*args, max_new_tokens=16, use_graph=False)
    assert graph == eager
    eos = obj.model.generation_config.eos_token_id       # the raw-template branch sets no eos override
    eos = [eos] if isinstance(eos, int) else list(eos or [])
    for i in range(3):
        enc, w = obj.decode_with_special_attention(question=args[0][i], paras=args[1][i], scores=args[2][i])
        with A.reweighting(obj.model, obj._bias(w, heads)), torch.no_grad():
            out = obj.model.generate(**enc, do_sample=False, max_new_tokens=16, output_scores=True,
                                     return_dict_in_generate=True, eos_token_id=eos)
        ref = out.sequences[0, enc["input_ids"].shape[1]:].tolist()
        got = obj.engine.generate([enc["input_ids"][0]], [w.cpu()], heads, max_new_tokens=16, eos_ids=eos)[0]
        gaps = [(s[0].float().topk(2).values[0] - s[0].float().topk(2).values[1]).item() for s in out.scores]
        for t in range(min(len(ref), len(got))):
            if ref[t] != got[t]:
                assert min(gaps[:t + 1]) < 0.05, (i, t, gaps[t])
                break

