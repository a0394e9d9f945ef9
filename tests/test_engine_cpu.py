"""Host-logic tests of the engine / IE sweep / transformers registration on the CPU.

cram_amd.ops is routed through tests/cpu_ops.py (fp32 CPU math, test-only) so
the plumbing around the kernels — fused weights, RoPE/RMSNorm/MLP op order,
variant construction of the head-batched sweep, last-layer row trimming, the
AttentionInterface registration and the per-call descriptor — is checked
against the reference's own golden outputs without a GPU.  The GPU suite runs
the same code paths on the HIP kernels.
"""
import gzip
import json
import os

import numpy as np
import pytest
import torch

from cram_amd import spans as S
import cram_amd.engine as engine_mod
from cram_amd.engine import CrAMEngine, DecodeSession
from cram_amd import sweep
from oracle import hook_ref
from tests import cpu_ops, parity
from tests import tiny_models as tm

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _gold(*names):
    rows = []
    for n in names:
        with gzip.open(os.path.join(GOLD, n), "rt") as f:
            rows += json.load(f)
    return rows


@pytest.fixture(scope="module")
def ie_gold():
    return _gold("tiny_ie.json.gz", "llama2_ie.json.gz")


@pytest.fixture(scope="module")
def nq():
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def tiny(tmp_path_factory):
    from transformers import AutoModelForCausalLM, AutoTokenizer
    root = str(tmp_path_factory.mktemp("m"))
    out = {}
    for k in ("llama3", "qwen2", "llama2"):
        p = tm.save_model(k, root)
        out[k] = (p, AutoTokenizer.from_pretrained(p), AutoModelForCausalLM.from_pretrained(p, dtype="auto").eval())
    return out


def _question(tok, path, rec, answer=True):
    paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
    ans = rec["wrong_answer"] if answer else ""
    _, enc, w, _ = S.encode(tok, path, rec["question"], paras, [0, 1, 1, 1, 1], ans)
    return enc["input_ids"], w


@pytest.mark.parametrize("kind", ["llama3", "qwen2", "llama2"])
def test_engine_logits_match_transformers(tiny, nq, kind):
    path, tok, model = tiny[kind]
    ids, w = _question(tok, path, nq[0])
    ids = ids[:, :300]
    from transformers import AutoModelForCausalLM
    f32 = AutoModelForCausalLM.from_pretrained(path, dtype=torch.float32).eval()
    with torch.no_grad():
        ref = model(input_ids=ids).logits[0, -5:].float()
        truth = f32(input_ids=ids).logits[0, -5:].float()
    eng = CrAMEngine.from_hf(model)
    assert eng.dtype == tm.dtype(kind)
    with cpu_ops.patched_ops():
        got = eng.logits(ids, last=5)[0].float()
    # bf16 noise floor: the engine must be as close to the fp32 model as transformers' own bf16 path is
    e_ref, e_got = (ref - truth).abs(), (got - truth).abs()
    assert e_got.mean() <= 1.5 * e_ref.mean() + 1e-3, (e_got.mean().item(), e_ref.mean().item())
    assert e_got.max() <= 2.0 * e_ref.max() + 1e-2, (e_got.max().item(), e_ref.max().item())


def test_oracle_ie_matches_reference_bitwise(tiny, nq, ie_gold):
    """The oracle's restated hook path reproduces the reference's cal_logits on the same CPU arithmetic."""
    path, tok, model = tiny["llama3"]
    g = [x for x in ie_gold if x["kind"] == "llama3" and x["variant"] == "bf16" and x["idx"] == 0][0]
    ids, w = _question(tok, path, nq[0])
    lw = hook_ref.log_weight(w)
    ans = torch.tensor(g["answer_ids"])
    grid = hook_ref.ie_grid(model, ids, lw, ans, layers=[0, 3], heads=[0, 1, 2, 3])
    np.testing.assert_array_equal(grid, np.asarray(g["ie"])[[0, 3]])


@pytest.fixture(scope="module")
def ie_truth():
    return _gold("tiny_ie_f32.json.gz", "llama2_ie_f32.json.gz")


def ie_tolerance_check(ie, ref, truth, agg=None, cpu=False):
    """Noise-floor criterion (written here once, used by the CPU and GPU suites).

    ref   = the reference's own bf16 (fp16 for Llama-2) run (fp32 logits), truth = the reference run on
    the float32 copy of the same weights.  The build must be as close to the truth as the
    reference's 16-bit arithmetic is (tests/parity.py: mean and max |ie-truth| within F x the reference's + A,
    F and A from the measured ratios); and every top-k set whose boundary gap in
    the truth exceeds 0.1 is identical for truth, ref and build.
    """
    ie, ref, truth = (np.asarray(x, dtype=np.float64) for x in (ie, ref, truth))
    e_ref, e_ie = np.abs(ref - truth), np.abs(ie - truth)
    a = agg if agg is not None else parity.Aggregate(cpu)
    a.ie_errors(e_ie, e_ref)
    if agg is None:                                 # a lone sample is its own aggregate
        a.check()
    flat_t = truth.reshape(-1)
    order = np.argsort(-flat_t, kind="stable")
    sv = flat_t[order]
    for k in range(1, flat_t.size):
        if sv[k - 1] - sv[k] > 0.1:
            top_t = set(order[:k])
            assert set(np.argsort(-ie.reshape(-1), kind="stable")[:k]) == top_t, k
            assert set(np.argsort(-ref.reshape(-1), kind="stable")[:k]) == top_t, k


@pytest.mark.parametrize("kind", ["llama3", "qwen2", "llama2"])
def test_sweep_matches_reference_ie(tiny, nq, ie_gold, ie_truth, kind):
    """Head-batched layer-suffix sweep vs the reference's 1 + L*H hooked forwards."""
    path, tok, model = tiny[kind]
    eng = CrAMEngine.from_hf(model)
    rows = [x for x in ie_gold if x["kind"] == kind and x["variant"] == "fp32"]
    agg = parity.Aggregate(cpu=True)
    for g in rows[:2]:
        t = [x for x in ie_truth if x["kind"] == kind and x["idx"] == g["idx"]][0]
        ids, w = _question(tok, path, nq[g["idx"]])
        ans = torch.tensor(g["answer_ids"])
        with cpu_ops.patched_ops():
            ie = sweep.ie_question(eng, ids[0], w[0], ans).double().numpy()
        ie_tolerance_check(ie, g["ie"], t["ie"], agg)
    agg.check()


def test_sweep_equals_unbatched_definition(tiny, nq):
    """Batched variants == one engine forward per (layer, head) with only that head biased (exact on CPU)."""
    from cram_amd.bias import CredibilityBias
    path, tok, model = tiny["qwen2"]
    eng = CrAMEngine.from_hf(model)
    ids, w = _question(tok, path, nq[2])
    ans = tok([nq[2]["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
    n = ans.numel()
    L, H = eng.spec.num_layers, eng.spec.num_heads
    with cpu_ops.patched_ops():
        def s(cb):
            hid = eng.forward_hidden(ids, cb, out_rows=n)[0]
            return (hid.float() @ eng.lm_head.float().T)[torch.arange(n), ans].sum().item()
        ori = s(None)
        un = np.array([[ori - s(CredibilityBias.build([w], {l: [h]}, L, H, "cpu")) for h in range(H)]
                       for l in range(L)])
        sw = sweep.ie_question(eng, ids[0], w[0], ans).double().numpy()
    np.testing.assert_allclose(sw, un, atol=2e-5)


def test_transformers_registration_plumbing(tiny, nq):
    """AttentionInterface "cram_hip" + descriptor == the hooked sdpa model (prefill + decode)."""
    from transformers import AutoModelForCausalLM
    from cram_amd import attention as A
    from cram_amd.bias import CredibilityBias
    path, tok, model = tiny["llama3"]
    A.register()
    m2 = AutoModelForCausalLM.from_pretrained(path, dtype="auto", attn_implementation=A.IMPL_NAME).eval()
    ids, w = _question(tok, path, nq[1], answer=False)
    ids = ids[:, :256]
    w = w[:, :256]
    heads = {0: [1], 1: [0, 3], 3: [2]}
    cb = CredibilityBias.build([w], heads, 4, 4, "cpu")
    hs = hook_ref.register_hooks(model, heads, hook_ref.log_weight(w))
    try:
        with torch.no_grad():
            ref = model(input_ids=ids).logits[0, -3:].float()
            ref_gen = model.generate(input_ids=ids, attention_mask=torch.ones_like(ids), do_sample=False,
                                     max_new_tokens=6)[0, 256:].tolist()
    finally:
        for h in hs:
            h.remove()
    with cpu_ops.patched_ops(), A.reweighting(m2, cb), torch.no_grad():
        got = m2(input_ids=ids).logits[0, -3:].float()
        gen = m2.generate(input_ids=ids, attention_mask=torch.ones_like(ids), do_sample=False,
                          max_new_tokens=6)[0, 256:].tolist()
    d = (got - ref).abs()            # bf16 noise floor of two attention implementations (sdpa vs eager: 0.10 / 0.019)
    assert d.max().item() < 0.15 and d.mean().item() < 0.025, (d.max().item(), d.mean().item())
    assert gen == ref_gen
    assert all(getattr(mod, "_cram_bias", None) is None for _, mod in A.attention_modules(m2))


def test_engine_batched_generate_matches_single(tiny, nq):
    """Ragged batch decode (per-row lengths + bias) == one-at-a-time decode, CPU stand-ins, no graph."""
    path, tok, model = tiny["llama3"]
    eng = CrAMEngine.from_hf(model)
    prompts, ws = [], []
    for i, L in ((0, 200), (1, 137), (2, 171)):
        ids, w = _question(tok, path, nq[i], answer=False)
        prompts.append(ids[0, :L])
        ws.append(w[:, :L])
    heads = {0: [1, 2], 2: [0]}
    with cpu_ops.patched_ops():
        both = eng.generate(prompts, ws, heads, max_new_tokens=5, use_graph=False)
        one = [eng.generate([p], [w], heads, max_new_tokens=5, use_graph=False)[0] for p, w in zip(prompts, ws)]
        # chunked packed prefill (chunks of <= 340 tokens: [200], [137, 171]) == one pass
        chunked, whole = DecodeSession(eng, prompts, ws, heads, 5), DecodeSession(eng, prompts, ws, heads, 5)
        chunked.prefill(max_rows=340)
        whole.prefill()
    # the batch's prompts share their chat-template opening: it is prefilled once and the suffixes attend over the
    # cache (cram_attn_prefill_varlen_cached); the single-prompt runs prefill whole prompts
    assert whole.prefix >= engine_mod.PREFIX_SHARE_MIN_ROWS, whole.prefix
    assert both == one
    # the decode step's projections on the split-K GEMM (cram_gemm_splitk; CRAM_DECODE_GEMM=all routes every
    # projection of the tiny shapes through it) == F.linear
    os.environ["CRAM_DECODE_GEMM"] = "all"
    try:
        with cpu_ops.patched_ops():
            sk = DecodeSession(eng, prompts, ws, heads, 5)
            assert all(sk.splits_gemm.values()), sk.splits_gemm
            allk = eng.generate(prompts, ws, heads, max_new_tokens=5, use_graph=False)
    finally:
        os.environ.pop("CRAM_DECODE_GEMM")
    assert allk == both
    os.environ["CRAM_DECODE_GEMM"] = "0"
    try:
        with cpu_ops.patched_ops():
            lib = eng.generate(prompts, ws, heads, max_new_tokens=5, use_graph=False)
            assert not any(DecodeSession(eng, prompts, ws, heads, 5).splits_gemm.values())
    finally:
        os.environ.pop("CRAM_DECODE_GEMM")
    assert lib == both
    assert chunked.tokens.tolist() == whole.tokens.tolist() == [r[0] for r in both]
    assert torch.equal(chunked.k_cache, whole.k_cache) and torch.equal(chunked.v_cache, whole.v_cache)
    # and against the hooked transformers model
    hs = hook_ref.register_hooks(model, heads, hook_ref.log_weight(ws[1]))
    try:
        with torch.no_grad():
            ref = model.generate(input_ids=prompts[1][None], attention_mask=torch.ones_like(prompts[1][None]),
                                 do_sample=False, max_new_tokens=5)[0, prompts[1].numel():].tolist()
    finally:
        for h in hs:
            h.remove()
    assert one[1] == ref


@pytest.mark.parametrize("kind", ["qwen2", "llama3"])
def test_engine_repetition_penalty_matches_generate(tiny, nq, kind):
    """Batched decode with the checkpoint's repetition penalty (Qwen chat generation_config ships 1.05; a strong
    1.5 here so it changes the ids) == transformers' greedy generate with the same penalty and the hook."""
    path, tok, model = tiny[kind]
    eng = CrAMEngine.from_hf(model)
    prompts, ws = [], []
    for i, L in ((3, 150), (4, 190)):
        ids, w = _question(tok, path, nq[i], answer=False)
        prompts.append(ids[0, :L])
        ws.append(w[:, :L])
    heads = {0: [0], 1: [1]}
    with cpu_ops.patched_ops():
        pen = eng.generate(prompts, ws, heads, max_new_tokens=12, use_graph=False, repetition_penalty=1.5)
        plain = eng.generate(prompts, ws, heads, max_new_tokens=12, use_graph=False)
    assert pen != plain                                   # the penalty is in effect
    for p, w, got in zip(prompts, ws, pen):
        hs = hook_ref.register_hooks(model, heads, hook_ref.log_weight(w))
        try:
            with torch.no_grad():
                ref = model.generate(input_ids=p[None], attention_mask=torch.ones_like(p[None]), do_sample=False,
                                     max_new_tokens=12, repetition_penalty=1.5)[0, p.numel():].tolist()
        finally:
            for h in hs:
                h.remove()
        assert got == ref


@pytest.mark.parametrize("kind", ["llama3", "qwen2"])
def test_engine_bad_words_match_generate(tiny, nq, kind):
    """Multi-token bad_words_ids (generate(bad_words_ids=...), re_weighting.py:128-129; transformers'
    NoBadWordsLogitsProcessor) in the batched engine == transformers' greedy generate with the same list and the hook.
    The list is built from the un-banned output so every kind of ban fires: a pair inside the generated ids, a pair
    that starts in the prompt, a triple, a single id, and a pair whose prefix never occurs."""
    path, tok, model = tiny[kind]
    eng = CrAMEngine.from_hf(model)
    prompts, ws = [], []
    for i, L in ((5, 160), (6, 185)):
        ids, w = _question(tok, path, nq[i], answer=False)
        prompts.append(ids[0, :L])
        ws.append(w[:, :L])
    heads = {0: [0], 1: [1]}
    with cpu_ops.patched_ops():
        plain = eng.generate(prompts, ws, heads, max_new_tokens=12, use_graph=False)
    g, p0 = plain[0], prompts[0]
    bad = [[g[2], g[3]], [int(p0[-1]), g[0]], [g[5], g[6], g[7]], [g[9]], [len(tok) - 1, g[1]]]
    with cpu_ops.patched_ops():
        got = eng.generate(prompts, ws, heads, max_new_tokens=12, use_graph=False, bad_words_ids=bad)
    assert got[0] != plain[0] and got[0][0] != g[0]                     # the prompt-spanning pair fired at once
    for p, w, row in zip(prompts, ws, got):
        hs = hook_ref.register_hooks(model, heads, hook_ref.log_weight(w))
        try:
            with torch.no_grad():
                ref = model.generate(input_ids=p[None], attention_mask=torch.ones_like(p[None]), do_sample=False,
                                     max_new_tokens=12, bad_words_ids=bad)[0, p.numel():].tolist()
        finally:
            for h in hs:
                h.remove()
        assert row == ref


def test_greedy_processors_guard(tiny):
    """run_RAG_batch takes the repetition penalty from generation_config and refuses processors it lacks."""
    from cram_amd.re_weighting import Re_Weighting_Strategy
    path, tok, model = tiny["qwen2"]
    obj = Re_Weighting_Strategy.__new__(Re_Weighting_Strategy)
    obj.model = model
    gc = model.generation_config
    old = (gc.repetition_penalty, gc.no_repeat_ngram_size)
    try:
        gc.repetition_penalty = 1.05
        assert obj._greedy_processors() == 1.05
        gc.no_repeat_ngram_size = 3
        with pytest.raises(NotImplementedError):
            obj._greedy_processors()
    finally:
        gc.repetition_penalty, gc.no_repeat_ngram_size = old


def test_fp32_truth_batched_grid_equals_per_unit(tiny, nq):
    """tests/fp32_llama.py: the per-layer batched float32 truth (used at the Llama-3-8B shape) equals one hooked
    float32 forward per unit up to float32 rounding."""
    from tests.fp32_llama import Fp32Llama
    path, tok, model = tiny["llama3"]
    eng = CrAMEngine.from_hf(model)
    ids, w = _question(tok, path, nq[5], answer=True)
    ids = ids[0, :180]
    w = w[0, :180]
    ans = ids[-3:]
    f32 = Fp32Llama(eng)
    bias = torch.log(w.float())
    units = [(l, h) for l in range(eng.spec.num_layers) for h in range(eng.spec.num_heads)]
    per = torch.tensor(f32.ie_units(ids, bias, ans, units), dtype=torch.float64).view(eng.spec.num_layers, -1)
    grid = f32.ie_grid(ids, bias, ans)
    assert per.abs().max() > 1e-3
    assert (grid - per).abs().max() < 1e-4 * max(1.0, per.abs().max().item())


def _ie_flops_by_enumeration(sp, T, n, p0):
    """Independent count of the IE sweep's algorithmic work (SURVEY §8(d) with the prefix skip): every weight matrix
    of every layer applied to the rows that need it, attention by summing each query row's visible keys."""
    D, F, d = sp.hidden, sp.intermediate, sp.head_dim
    mats = {"q": (sp.q_size, D), "k": (sp.kv_size, D), "v": (sp.kv_size, D), "o": (D, sp.q_size),
            "gate": (F, D), "up": (F, D), "down": (D, F)}

    def gemm(names, rows):
        return sum(2 * mats[m][0] * mats[m][1] * rows for m in names)

    memo = {}

    def attn(q_rows):                         # query rows at absolute positions q_rows, causal over keys 0..i
        if q_rows not in memo:
            memo[q_rows] = sum(4 * d * sp.num_heads * (i + 1) for i in q_rows)
        return memo[q_rows]

    L, H = sp.num_layers, sp.num_heads
    everything, rest = list(mats), ["o", "gate", "up", "down"]
    suffix, answer = range(p0, T), range(T - n, T)
    f = 0
    for l in range(L):                         # the un-hooked forward
        if l < L - 1:
            f += gemm(everything, T) + attn(range(T))
        else:                                  # K / V of every row, the rest for the answer rows
            f += gemm(["k", "v"], T) + gemm(["q"] + rest, n) + attn(answer)
    for l in range(L):                         # per hooked layer: the all-heads-biased attention, then H variants
        rows = answer if l == L - 1 else suffix
        f += attn(rows)
        for _h in range(H):
            f += gemm(rest, len(rows))
            for l2 in range(l + 1, L):
                if l2 == L - 1:
                    f += gemm(["k", "v"], len(suffix)) + gemm(["q"] + rest, n) + attn(answer)
                else:
                    f += gemm(everything, len(suffix)) + attn(suffix)
    return f


def test_sweep_flops_accounting():
    """sweep_flops (the step roofline's numerator) equals an independent enumeration of SURVEY §8(d)'s work with the
    prefix skip (32 variants, the last layer's q / attention / MLP on the answer rows); what the sweep executes on top
    (the un-perturbed variant, pad rows) is sweep_flops_executed, reported beside it."""
    from cram_amd.engine import ModelSpec
    sp = ModelSpec.llama3_8b()
    for T, n, p0 in ((904, 4, 25), (907, 3, 0), (962, 5, 37)):
        f = sweep.sweep_flops(sp, T, n, p0)
        assert f == pytest.approx(_ie_flops_by_enumeration(sp, T, n, p0), rel=1e-12)
        ex = sweep.sweep_flops_executed(sp, T, n, p0)
        # the 33rd variant adds ~1/32 of the variant work; pad rows at most +2048 GEMM rows per batch
        assert 1.025 * f < ex < 1.12 * f
        assert sweep.sweep_flops_executed(sp, T, n, p0, base_variant=False) < ex
    small = ModelSpec(3, 256, 4, 2, 128, 512, 1000, 1e-5, False, "llama")
    assert sweep.sweep_flops(small, 97, 3, 11) == pytest.approx(_ie_flops_by_enumeration(small, 97, 3, 11), rel=1e-12)
    assert sweep.sweep_flops(small, 97, 3, 11, layers=[2]) < sweep.sweep_flops(small, 97, 3, 11, layers=[0])
    ref_fwd = 2 * (6.98e9 + 0.525e9) * 904          # one reference-style full forward
    assert 0.3 * 1025 * ref_fwd < sweep.sweep_flops(sp, 904, 4) < 0.6 * 1025 * ref_fwd


@pytest.mark.parametrize("family", ["llama", "qwen2"])
def test_cpu_baseline_model_matches_engine(family):
    """bench.py's CPU baseline runs the same network as the engine (weights copied back into transformers; the
    Qwen2 family with its q/k/v biases), and its decode sample runs the reference's hooked generate."""
    from cram_amd.engine import ModelSpec
    from oracle import cpu_baseline
    sp = ModelSpec(2, 256, 4, 2, 128, 512, 1000, 1e-5, family == "qwen2", family)
    eng = CrAMEngine.random(sp, torch.device("cpu"), seed=3, std=0.05)
    model = cpu_baseline.hf_model_from_engine(eng)
    ids = torch.randint(0, 1000, (1, 77), generator=torch.Generator().manual_seed(77))
    w = torch.ones((1, 77), dtype=torch.float16)
    w[:, 10:30] = 0
    with torch.no_grad():
        ref = model(input_ids=ids).logits[0, -3:].float()
    with cpu_ops.patched_ops():
        got = eng.logits(ids, last=3)[0].float()
    assert (got - ref).abs().max() < 0.1 and (got - ref).abs().mean() < 0.02
    r = cpu_baseline.time_ie_units(model, ids, w, torch.tensor([5, 6]), [(0, 1), (1, 2)])
    assert r["units"] == 2 and r["units_per_s"] > 0 and all(np.isfinite(r["ie"]))
    d = cpu_baseline.time_decode(model, ids, w, {0: [1], 1: [0, 3]}, new_tokens=100, sampled_steps=3)
    assert d["sampled_steps"] == 3 and d["prefill_s"] > 0 and d["heads"] == 3
    assert d["question_s"] == pytest.approx(d["prefill_s"] + 99 * d["step_s"]["median"])
    # the long-prompt form: the first layer only, times scaled by L / k; the model is whole again afterwards
    d1 = cpu_baseline.time_decode(model, ids, w, {0: [1], 1: [0, 3]}, new_tokens=100, sampled_steps=2, layers=1)
    assert (d1["layers_run"], d1["layers"], d1["heads"]) == (1, 2, 1)
    assert len(model.model.layers) == 2 and model.config.num_hidden_layers == 2
    # the hooked greedy ids of the sample equal the engine's batched decode with the same bias, up to the first
    # near-tie (top-2 logit gap < 0.05: two bf16 evaluations of the same network may pick either)
    hs = hook_ref.register_hooks(model, {0: [1], 1: [0, 3]}, hook_ref.log_weight(w))
    try:
        with torch.no_grad():
            out = model.generate(input_ids=ids, attention_mask=torch.ones_like(ids), do_sample=False,
                                 max_new_tokens=4, min_new_tokens=4, pad_token_id=0, output_scores=True,
                                 return_dict_in_generate=True)
    finally:
        for h in hs:
            h.remove()
    ref_ids = out.sequences[0, 77:].tolist()
    gaps = [float(torch.topk(sc[0].float(), 2).values.diff().abs()) for sc in out.scores]
    with cpu_ops.patched_ops():
        got_ids = eng.generate([ids[0]], [w], {0: [1], 1: [0, 3]}, max_new_tokens=4, use_graph=False)[0]
    assert len(got_ids) == len(ref_ids) == 4
    for t in range(4):
        if got_ids[t] != ref_ids[t]:
            assert min(gaps[:t + 1]) < 0.05, (t, got_ids, ref_ids, gaps)
            break


def test_sweep_prefix_skip_is_exact(tiny, nq):
    """Rows before the first biased key are identical in every variant: computing only the suffix (K/V of
    the prefix from the baseline forward) gives the same IE as recomputing every row."""
    path, tok, model = tiny["llama3"]
    eng = CrAMEngine.from_hf(model)
    ids, w = _question(tok, path, nq[0])
    ans = tok([nq[0]["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
    from cram_amd.bias import CredibilityBias
    p0 = sweep.first_biased_row(CredibilityBias.build([w], {}, 1, 1, "cpu").bias, w.shape[-1])
    assert 0 < p0 < ids.shape[1] - ans.numel()
    with cpu_ops.patched_ops():
        a = sweep.ie_question(eng, ids[0], w[0], ans, skip_prefix=True)
        b = sweep.ie_question(eng, ids[0], w[0], ans, skip_prefix=False)
    assert torch.equal(a, b)
    T = ids.shape[1]
    assert sweep.sweep_flops(eng.spec, T, ans.numel(), p0) < sweep.sweep_flops(eng.spec, T, ans.numel())



@pytest.mark.parametrize("kind", ["llama3", "qwen2"])
def test_sweep_grouped_batches_equal_per_layer_batches(tiny, nq, kind, monkeypatch):
    """group_variants (consecutive swept layers in one growing batch, each layer's batch joining after its attention)
    computes the variants layer_variants does: the same IE grid as one batch per layer, with and without the prefix
    skip, for every grouping (on the GPU's row-independent kernels bit for bit, tests/test_fullsize_ie_gpu.py)."""
    path, tok, model = tiny[kind]
    eng = CrAMEngine.from_hf(model)
    ids, w = _question(tok, path, nq[1])
    ans = tok([nq[1]["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
    assert sweep.sweep_groups(range(eng.spec.num_layers), eng.spec.num_layers, 2)[-1] == [eng.spec.num_layers - 1]
    with cpu_ops.patched_ops():
        for skip in (True, False):
            monkeypatch.setattr(sweep, "SWEEP_GROUP", 1)
            a = sweep.ie_question(eng, ids[0], w[0], ans, skip_prefix=skip)
            for g in (2, 3):
                monkeypatch.setattr(sweep, "SWEEP_GROUP", g)
                b = sweep.ie_question(eng, ids[0], w[0], ans, skip_prefix=skip)
                assert (a - b).abs().max() <= 1e-3 * max(1.0, float(a.abs().max())), (skip, g, (a - b).abs().max())


def test_padded_rows_table():
    """GEMM row padding: a multiple of 256, never fewer rows, at most +2048 with the Llama-3-8B table; other
    shapes (and no spec) keep plain 256-row rounding."""
    from cram_amd.engine import ModelSpec, padded_rows
    sp = ModelSpec.llama3_8b()
    for M in list(range(1, 3000, 97)) + list(range(16000, 41000, 131)) + [70000]:
        p = padded_rows(M, sp)
        assert p % 256 == 0 and M <= p <= -(-M // 256) * 256 + 2048
        assert padded_rows(M) == -(-M // 256) * 256
        assert padded_rows(M, ModelSpec.qwen2_7b()) == padded_rows(M)
    assert padded_rows(32400, sp) == 32768        # measured: 32768 rows (8 x 4096) run cheaper than 32512


def test_decode_split_plan():
    """K ranges of the decode step's long-K down_proj (engine.decode_splits): column tiles toward 128 workgroups up to
    512 rows (8 ranges for Llama-3 at 256 / 500 rows, 14 at config 5's 129), the row tiles counted beyond 512 rows
    toward one workgroup per CU (4 ranges at 1,000 rows for Llama-3 and Qwen2-7B), the library past 1,024 rows; the
    short-K projections stay on the library."""
    ds = engine_mod.decode_splits
    assert [ds(4096, 14336, r) for r in (129, 256, 500, 512, 1000, 1024, 1025)] == [14, 8, 8, 8, 4, 4, 0]
    assert ds(3584, 18944, 1000) == 4 and ds(3584, 18944, 500) == 8
    assert ds(6144, 4096, 1000) == 0 and ds(4096, 4096, 1000) == 0 and ds(28672, 4096, 1000) == 0
