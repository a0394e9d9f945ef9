"""The decode step the bench times, pinned as a whole.

bench.py's decode legs run `CrAMEngine.generate` with the routing the engine picks from the batch size: config 2
(Llama-3-8B, NQ-1000 on one GPU = two batches of 500 rows) and config 5 (20 retrieved docs, ~8.3k-token prompts, 128
rows from the KV budget; also every GPU's share of NQ-1000 at 8 GPUs).  Kernel-level tests cover each piece against fp32; here the routed step is checked end to
end, at Llama-3-8B's widths (D 4096, 32 / 8 heads of 128, FFN 14336, vocab 128256; two layers of random weights --
the depth is irrelevant to the routing, the widths are not), on the bench's own inputs (rebuilt NQ prompts through the
Llama-3 chat template, ideal scores, the nq/llama3 selected heads of layers 0-1), against

  (i)  the same engine with CRAM_DECODE_GEMM=0: every decode projection on the library GEMM (hipBLASLt + the
       separate SiLU-mul), nothing of the decode routing left -- greedy ids equal up to the first near-tie;
  (ii) the transformers drop-in (the engine's weights in a LlamaForCausalLM on the cram_hip AttentionInterface,
       model.generate at batch 1, re_weighting.py:115-138) on a few of the same rows -- ids equal up to the
       drop-in's first near-tie.

A divergence is accepted only at a near-tie: the top-2 logit gap of the diverging step, measured by a teacher-forced
engine forward of the prompt and the common prefix with the same credibility bias, below NEAR_TIE.
"""
import gzip
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAME = "Meta-Llama-3-8B-Instruct"          # the chat template branch of the Llama-3 family (spans.encode)
NEAR_TIE = 0.1                              # top-2 logit gap (teacher-forced) below which greedy ids may differ


@pytest.fixture(scope="module")
def l3w(gpu_device):
    """A two-layer model at Llama-3-8B's widths, random init as the bench's (CrAMEngine.random)."""
    from transformers import AutoTokenizer
    from cram_amd.engine import CrAMEngine, ModelSpec
    sp = ModelSpec(2, 4096, 32, 8, 128, 14336, 128256, 1e-5, False, "llama")
    eng = CrAMEngine.random(sp, gpu_device, seed=11, rope_theta=500000.0)
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3"))
    heads = json.load(open(os.path.join(REPO, "data", "selected_heads.json")))["nq__llama3"]["heads"]
    heads = {l: v for l, v in heads.items() if int(l) < sp.num_layers}
    assert heads, "no selected heads in layers 0-1"
    yield eng, tok, heads
    del eng
    torch.cuda.empty_cache()


def _nq(n, long_context=False):
    from cram_amd import scores
    with gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8") as f:
        data = json.load(f)
    qs, ps, ss = [], [], []
    for i in range(n):
        if long_context:
            import bench
            paras, sc = bench.long_context_paras(data, i)
        else:
            paras, sc = scores.assemble(data[i], ideal=True, ideal_score=1)
        qs.append(data[i]["question"])
        ps.append(paras)
        ss.append(sc)
    return qs, ps, ss


def _encode(tok, n, long_context=False):
    from cram_amd import spans
    encs = spans.encode_batch(tok, NAME, *_nq(n, long_context))
    return [ids for ids, _, _ in encs], [w for _, w, _ in encs]


def _gap(eng, heads, prompt, w, prefix):
    """Top-2 logit gap of the next token after prompt + prefix (teacher-forced engine forward, same bias)."""
    from cram_amd.bias import CredibilityBias
    sp = eng.spec
    ids = torch.cat([prompt.cpu(), torch.tensor(prefix, dtype=prompt.dtype)]).view(1, -1).to(eng.device)
    cb = CredibilityBias.build([w.reshape(1, -1)], heads, sp.num_layers, sp.num_heads, eng.device, eng.dtype)
    lg = eng.logits(ids, cb, last=1)[0, -1].float()
    return float(torch.topk(lg, 2).values.diff().abs())


def _compare(eng, heads, prompts, ws, a, b, what):
    """Rows of two greedy runs: equal, or equal up to a step whose (teacher-forced) top-2 gap is a near-tie."""
    equal_rows = tokens = 0
    worst = 0.0
    for r, (x, y) in enumerate(zip(a, b)):
        t = next((i for i in range(min(len(x), len(y))) if x[i] != y[i]), None)
        if t is None:
            equal_rows += 1
            tokens += len(x)
            continue
        g = _gap(eng, heads, prompts[r], ws[r], x[:t])
        worst = max(worst, g)
        assert g < NEAR_TIE, f"{what}: row {r} diverges at step {t} with a top-2 gap of {g:.4f}"
        tokens += t
    n = sum(len(x) for x in a)
    print(f"\n{what}: {equal_rows}/{len(a)} rows equal, {tokens}/{n} tokens before any divergence, "
          f"largest gap at a divergence {worst:.4f}")
    return equal_rows, tokens / n


def _dropin_ids(eng, heads, prompts, ws, rows, new):
    """model.generate at batch 1 through the cram_hip AttentionInterface (the drop-in path), with its per-step
    scores; the engine's weights in a transformers LlamaForCausalLM."""
    from cram_amd import attention as A
    from cram_amd.bias import CredibilityBias
    from oracle.cpu_baseline import hf_model_from_engine
    sp = eng.spec
    A.register()
    model = hf_model_from_engine(eng).to(eng.device)
    model.set_attn_implementation(A.IMPL_NAME)
    out = {}
    try:
        for r in rows:
            ids = prompts[r].view(1, -1).to(eng.device)
            cb = CredibilityBias.build([ws[r].reshape(1, -1)], heads, sp.num_layers, sp.num_heads, eng.device,
                                       eng.dtype)
            with A.reweighting(model, cb), torch.no_grad():
                g = model.generate(input_ids=ids, attention_mask=torch.ones_like(ids), do_sample=False,
                                   max_new_tokens=new, min_new_tokens=new, pad_token_id=0, output_scores=True,
                                   return_dict_in_generate=True)
            gaps = [float(torch.topk(s[0].float(), 2).values.diff().abs()) for s in g.scores]
            out[r] = (g.sequences[0, ids.shape[1]:].tolist(), gaps)
    finally:
        del model
        torch.cuda.empty_cache()
    return out


def _check_dropin(engine_rows, dropin):
    compared = 0
    for r, (ref, gaps) in dropin.items():
        got = engine_rows[r]
        for t in range(min(len(ref), len(got))):
            if ref[t] != got[t]:
                assert min(gaps[:t + 1]) < 0.05, (r, t, gaps[:t + 1])
                break
            compared += 1
    return compared


def _routing(eng, prompts, ws, heads, new):
    from cram_amd.engine import DecodeSession
    s = DecodeSession(eng, prompts, ws, heads, new)
    r = dict(s.splits_gemm, mlp_w4=s.mlp_w4, lm_w4=s.lm_w4, attn_splits=s.splits, B=s.B, small=dict(s.small))
    del s
    return r


@pytest.mark.parametrize("n", [500, 1000])
def test_config2_step_at_500_rows(l3w, monkeypatch, n):
    """Config 2's timed batch -- round 6: NQ-1000 in ONE batch of 1000 rows (bench --decode-batch 1024, KV cache in
    0.68 of HBM; 81.8 vs 79.5 questions/s for two batches of 500, profiles/r06/decode_b*.json), and the 500-row batch
    of rounds 3-5: gate/up + SiLU-mul and lm_head on gemm_w4_kernel inside the captured step graph, down_proj over 8 K
    ranges at 500 rows and 4 at 1000 (the row tiles counted beyond 512 rows: one workgroup per CU), q/k/v / o_proj on
    the library; the shared prompt opening read from cache row 0 by the decode attention."""
    from cram_amd import engine as E
    eng, tok, heads = l3w
    prompts, ws = _encode(tok, n)
    new = 12
    rt = _routing(eng, prompts, ws, heads, new)
    assert (rt["mlp_w4"] and rt["lm_w4"] and rt["down"] == {500: 8, 1000: 4}[n] and n <= E.DECODE_GEMM_MAX_ROWS
            and rt["qkv"] == 0 and rt["o"] == 0 and rt["gu"] == 0 and not rt["small"]), rt
    got = eng.generate(prompts, ws, heads, max_new_tokens=new, use_graph=True, stop_on_eos=False)
    assert eng.generate(prompts[:3], ws[:3], heads, max_new_tokens=new, use_graph=False, stop_on_eos=False) is not None
    monkeypatch.setenv("CRAM_DECODE_GEMM", "0")
    rl = _routing(eng, prompts, ws, heads, new)
    assert not (rl["mlp_w4"] or rl["lm_w4"] or rl["down"] or rl["qkv"] or rl["o"] or rl["gu"] or rl["small"]), rl
    lib = eng.generate(prompts, ws, heads, max_new_tokens=new, use_graph=True, stop_on_eos=False)
    monkeypatch.delenv("CRAM_DECODE_GEMM")
    rows, frac = _compare(eng, heads, prompts, ws, got, lib, "config 2 routed vs library step")
    assert frac >= 0.5 and rows >= len(got) // 4
    dropin = _dropin_ids(eng, heads, prompts, ws, [0, n // 2, n - 1], new)
    assert _check_dropin(got, dropin) >= 6


def test_config5_step_at_128_rows(l3w, monkeypatch):
    """Config 5's batch (128 rows of ~8.3k tokens, the KV budget in whole 64-row groups): q/k/v, o_proj and down_proj
    on cram_gemm_small with K split over 4 / 8 / 8 ranges, lm_head on gemm_w4_kernel, 2 attention splits (rows of
    >= 4k keys), gate/up on the library (the 4-wave kernel loses at this row count)."""
    eng, tok, heads = l3w
    prompts, ws = _encode(tok, 128, long_context=True)
    assert 7000 < sum(p.numel() for p in prompts) / len(prompts) < 10000
    new = 8
    rt = _routing(eng, prompts, ws, heads, new)
    assert (rt["small"] == {"qkv": 4, "o": 8, "down": 8} and rt["lm_w4"] and not rt["mlp_w4"] and rt["gu"] == 0
            and rt["attn_splits"] >= 2), rt
    got = eng.generate(prompts, ws, heads, max_new_tokens=new, use_graph=True, stop_on_eos=False)
    monkeypatch.setenv("CRAM_DECODE_GEMM", "0")
    lib = eng.generate(prompts, ws, heads, max_new_tokens=new, use_graph=True, stop_on_eos=False)
    monkeypatch.delenv("CRAM_DECODE_GEMM")
    rows, frac = _compare(eng, heads, prompts, ws, got, lib, "config 5 routed vs library step")
    assert frac >= 0.5 and rows >= len(got) // 4
    dropin = _dropin_ids(eng, heads, prompts, ws, [0, 127], new)
    assert _check_dropin(got, dropin) >= 4


def test_shared_prefix_prefill_at_llama3_widths(l3w, monkeypatch):
    """The batch's common chat-template opening prefilled once, the suffixes over the cache
    (cram_attn_prefill_varlen_cached), against whole-prompt prefill (CRAM_PREFIX_SHARE off): the prefix's K/V equal
    the whole-prompt prefill's within bf16 GEMM-order noise, and the greedy ids agree up to near-ties."""
    from cram_amd import engine as E
    eng, tok, heads = l3w
    prompts, ws = _encode(tok, 64)
    new = 12
    s = E.DecodeSession(eng, prompts, ws, heads, new)
    s.prefill()
    p = s.prefix
    assert p >= E.PREFIX_SHARE_MIN_ROWS, p
    monkeypatch.setattr(E, "PREFIX_SHARE", False)
    s0 = E.DecodeSession(eng, prompts, ws, heads, new)
    s0.prefill()
    assert s0.prefix == 0
    for c, c0 in ((s.k_cache, s0.k_cache), (s.v_cache, s0.v_cache)):
        a, b = c[:, :, :, :p].float(), c0[:, :, :, :p].float()
        # layer 0: the prefix runs the packed prefill's own GEMM kernels (row-independent): bit-equal
        assert torch.equal(c[0, :, :, :p], c0[0, :, :, :p])
        # above it only the attention kernel's 32-row blocks fall differently (prefix alone vs whole prompt)
        d = (a - b).abs()
        eq = float((a == b).float().mean())
        print(f"\nprefix K/V vs whole-prompt prefill: max |diff| {d.max():.3e} (max |x| {b.abs().max():.2f}), "
              f"mean |diff| {d.mean():.3e}, equal {eq:.4f}")
        # measured: max 3.1e-2 (one bf16 ulp at |x| ~ 6), 98.4 % of the elements equal (profiles/r06/)
        assert d.max() <= 0.01 * b.abs().max() + 0.01, d.max()
        assert eq >= 0.95, eq
    whole = eng.generate(prompts, ws, heads, max_new_tokens=new, use_graph=True, stop_on_eos=False)
    monkeypatch.setattr(E, "PREFIX_SHARE", True)
    shared = eng.generate(prompts, ws, heads, max_new_tokens=new, use_graph=True, stop_on_eos=False)
    rows, frac = _compare(eng, heads, prompts, ws, shared, whole, "shared-prefix vs whole-prompt prefill")
    assert frac >= 0.5 and rows >= len(shared) // 4
