"""End-to-end GPU parity of the drop-in API on the tiny models (HIP kernels, no CPU fallback).

Against vectors the reference itself produced (tests/golden/gen_golden.py):
  * decode_with_special_attention: ids + fp16 weights bit-exact;
  * Find_Best_Heads.cal_logits: IE within the bf16 noise floor of the reference
    (criterion in tests/test_engine_cpu.py::ie_tolerance_check) and identical
    top-k sets wherever the truth has a gap > 0.1;
  * run_RAG_with_attention_weighting: greedy ids equal to the reference's up to the
    first step whose top-2 logit gap is below 0.05 (a near-tie bf16 noise can flip);
  * engine batched / graph-replayed decode == the transformers drop-in decode;
  * batched IE sweep == one forward per (layer, head) on the same kernels.
"""
import gzip
import json
import os

import numpy as np
import pytest
import torch

from tests import parity
from tests import tiny_models as tm
from tests.test_engine_cpu import ie_tolerance_check

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with gzip.open(os.path.join(GOLD, name), "rt", encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def nq():
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def paths(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("tiny"))
    return {k: tm.save_model(k, root) for k in ("llama3", "qwen2", "qwen2_gqa7")}


# golden files per kind: (IE grids, IE of the float32 copy, answer log-probs); the GQA-7 kind has its own
def _gold_files(kind):
    if kind == "qwen2_gqa7":
        return "qwen2_gqa7_ie.json.gz", "qwen2_gqa7_ie_f32.json.gz", "qwen2_gqa7_logprobs.json.gz"
    return "tiny_ie.json.gz", "tiny_ie_f32.json.gz", "logprobs.json.gz"


def _first3(agg_all, kind, ie_err, ref_err, idx):
    """The original three Qwen2 questions (idx 0-2) as their own logged aggregate."""
    if kind == "qwen2" and idx < 3:
        agg_all.setdefault("first3", parity.Aggregate(label="qwen2 idx 0-2")).ie_errors(ie_err, ref_err,
                                                                                       subset="qwen2 idx 0-2", idx=idx)


@pytest.fixture(scope="module")
def fbh(paths, gpu_device):
    from cram_amd.re_weighting import Find_Best_Heads
    return {k: Find_Best_Heads(model_name=p) for k, p in paths.items()}


def test_spans_on_device(fbh):
    rows = _load("spans.json.gz")
    for r in rows[::7]:
        obj = fbh[r["kind"]]
        enc, w = obj.decode_with_special_attention(question=r["question"], paras=r["paras"], scores=r["scores"],
                                                   answer=r["answer"])
        assert enc["input_ids"].is_cuda and w.dtype == torch.float16
        assert enc["input_ids"][0].tolist() == r["input_ids"]
        assert w[0].float().tolist() == r["weight"]


def _sub_errors(ie, ref, truth):
    ie, ref, truth = (np.asarray(x, dtype=np.float64) for x in (ie, ref, truth))
    return np.abs(ie - truth), np.abs(ref - truth)


@pytest.mark.parametrize("kind", ["llama3", "qwen2", "qwen2_gqa7"])
def test_cal_logits_matches_reference(fbh, nq, kind):
    f_ie, f_truth, _ = _gold_files(kind)
    gold = [x for x in _load(f_ie) if x["kind"] == kind and x["variant"] == "fp32"]
    truth = {x["idx"]: x["ie"] for x in _load(f_truth) if x["kind"] == kind}
    obj = fbh[kind]
    agg, sub = parity.Aggregate(), {}
    for g in gold:
        rec = nq[g["idx"]]
        ie = obj.cal_logits(question=rec["question"], paras=rec["ori_fake"] + rec["reranked_dense_ctxs"],
                            scores=[0, 1, 1, 1, 1], wrong_answer=rec["wrong_answer"])
        assert isinstance(ie, list) and len(ie) == obj.model_num_hidden_layers
        assert all(isinstance(v, float) for v in ie[0])
        ie_tolerance_check(ie, g["ie"], truth[g["idx"]], agg)
        _first3(sub, kind, *_sub_errors(ie, g["ie"], truth[g["idx"]]), g["idx"])
    if kind == "qwen2_gqa7":                         # >= 6 questions whose IE is not identically 0
        assert agg.informative("ie_max") >= 6
    agg.check()
    for a in sub.values():
        a.log_aggregates()


@pytest.mark.parametrize("kind", ["llama3", "qwen2", "qwen2_gqa7"])
def test_cal_logits_bf16_logits_match_reference(fbh, nq, kind):
    """round_logits=True (each answer logit rounded to the model dtype, as transformers 5.15 returns them) against
    the reference run under the same convention (G4 'bf16' variant, re_weighting.py:159-160,170), same bar."""
    f_ie, f_truth, _ = _gold_files(kind)
    gold = [x for x in _load(f_ie) if x["kind"] == kind and x["variant"] == "bf16"]
    truth = {x["idx"]: x["ie"] for x in _load(f_truth) if x["kind"] == kind}
    assert gold
    obj = fbh[kind]
    agg, sub = parity.Aggregate(), {}
    for g in gold:
        rec = nq[g["idx"]]
        ie = obj.cal_logits_tensor(question=rec["question"], paras=rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                   scores=[0, 1, 1, 1, 1], wrong_answer=rec["wrong_answer"], round_logits=True)
        ie = ie.double().cpu().numpy()
        ie_tolerance_check(ie, g["ie"], truth[g["idx"]], agg)
        _first3(sub, kind, *_sub_errors(ie, g["ie"], truth[g["idx"]]), g["idx"])
    if kind == "qwen2_gqa7":
        assert agg.informative("ie_max") >= 6
    agg.check()
    for a in sub.values():
        a.log_aggregates()


def test_qwen2_ie_against_reference_executions(fbh, paths, nq, gpu_device):
    """The tiny Qwen2's first three questions (our IE max error 1.6-1.9x the fixture's on idx 0 and 2).
    The fixture is ONE execution of the reference code (CPU, transformers sdpa); other valid bf16 executions of the
    same unmodified algorithm -- the dense-mask hook on transformers' GPU sdpa and eager attention (oracle/hook_ref.py,
    bit-exact to re_weighting.py on CPU) -- land 0.07-0.12 from the float32 truth on those questions, where the CPU
    sdpa draw landed 0.036-0.039 (tools/ie_noise_probe.py, profiles/r06/ie_noise.jsonl).  The reference's own error
    is therefore measured here as the mean over the three executions, and ours (the sweep) must stay within 1.3x of it
    over the three questions, mean and max of |IE - truth| (the original per-fixture bar is
    test_cal_logits_matches_reference's)."""
    from transformers import AutoModelForCausalLM
    from oracle import hook_ref
    gold = {x["idx"]: x["ie"] for x in _load("tiny_ie.json.gz") if x["kind"] == "qwen2" and x["variant"] == "fp32"}
    truth = {x["idx"]: np.array(x["ie"]) for x in _load("tiny_ie_f32.json.gz") if x["kind"] == "qwen2"}
    obj = fbh["qwen2"]
    models = [AutoModelForCausalLM.from_pretrained(paths["qwen2"], dtype=torch.bfloat16,
                                                   attn_implementation=impl).eval().to(gpu_device)
              for impl in ("sdpa", "eager")]
    tot = {"ours_mean": 0.0, "ours_max": 0.0, "ref_mean": 0.0, "ref_max": 0.0}
    for i in range(3):
        rec = nq[i]
        paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
        ours = np.array(obj.cal_logits(question=rec["question"], paras=paras, scores=[0, 1, 1, 1, 1],
                                       wrong_answer=rec["wrong_answer"]))
        enc, w = obj.decode_with_special_attention(question=rec["question"], paras=paras, scores=[0, 1, 1, 1, 1],
                                                   answer=rec["wrong_answer"])
        ans = obj.answer_ids(rec["wrong_answer"]).to(gpu_device)
        runs = [np.array(gold[i])]
        for m in models:
            h = m.lm_head.register_forward_hook(
                lambda mod, a, o: torch.nn.functional.linear(a[0].float(), mod.weight.float()))
            try:
                runs.append(hook_ref.ie_grid(m, enc["input_ids"], hook_ref.log_weight(w).to(gpu_device), ans))
            finally:
                h.remove()
        t = truth[i]
        e_ref = [np.abs(r - t) for r in runs]
        e_o = np.abs(ours - t)
        tot["ours_mean"] += e_o.mean()
        tot["ours_max"] += e_o.max()
        tot["ref_mean"] += float(np.mean([e.mean() for e in e_ref]))
        tot["ref_max"] += float(np.mean([e.max() for e in e_ref]))
        parity.record("ie_max", e_o.max(), float(np.mean([e.max() for e in e_ref])), idx=i,
                      reference_kind="mean of 3 executions", executions=[float(e.max()) for e in e_ref])
    for fam in ("mean", "max"):
        parity.record(f"ie_{fam}_aggregate", tot[f"ours_{fam}"], tot[f"ref_{fam}"], samples=3,
                      reference_kind="mean of 3 executions")
        assert tot[f"ours_{fam}"] <= 1.3 * tot[f"ref_{fam}"], (fam, tot)


def test_cal_logits_deterministic(fbh, nq):
    rec = nq[3]
    args = dict(question=rec["question"], paras=rec["ori_fake"] + rec["reranked_dense_ctxs"], scores=[0, 1, 1, 1, 1],
                wrong_answer=rec["wrong_answer"])
    a = fbh["llama3"].cal_logits_tensor(**args)
    b = fbh["llama3"].cal_logits_tensor(**args)
    assert torch.equal(a, b)


def test_top_k_ranking_over_questions(fbh, nq):
    """Mean-IE ranking over the golden questions: identical top-k sets at well-separated k."""
    from cram_amd.heads import rank_heads
    gold = [x for x in _load("tiny_ie.json.gz") if x["kind"] == "llama3" and x["variant"] == "fp32"]
    truth = [x["ie"] for x in _load("tiny_ie_f32.json.gz") if x["kind"] == "llama3"]
    ours = []
    for g in gold:
        rec = nq[g["idx"]]
        ours.append(fbh["llama3"].cal_logits(question=rec["question"],
                                             paras=rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                             scores=[0, 1, 1, 1, 1], wrong_answer=rec["wrong_answer"]))
    r_t = rank_heads(truth)
    r_o = rank_heads(ours)
    vals = [v for v, _ in r_t]
    for k in range(1, len(vals)):
        if vals[k - 1] - vals[k] > 0.05:
            assert {lh for _, lh in r_t[:k]} == {lh for _, lh in r_o[:k]}, k


def _drop_in(paths, kind, heads, gpu_device):
    from cram_amd.re_weighting import Re_Weighting_Strategy
    return Re_Weighting_Strategy(model_name=paths[kind], layers_to_be_modified=dict(heads), bad_words_ids=[])


def _gaps(scores):
    g = []
    for s in scores:
        top = torch.topk(s[0].float(), 2).values
        g.append((top[0] - top[1]).item())
    return g


@pytest.mark.parametrize("case", [0, 1, 2])
def test_generate_matches_reference(paths, nq, gpu_device, case):
    gold = _load("generate.json.gz")
    kinds = [("llama3", {0: [1], 1: [0, 3], 3: [2]}), ("llama3", {}), ("qwen2", {1: [0]})]
    kind, heads = kinds[case]
    rows = [g for g in gold if g["kind"] == kind and g["heads"] == {str(k): v for k, v in heads.items()}]
    obj = _drop_in(paths, kind, heads, gpu_device)
    from cram_amd import attention as A
    for g in rows[:2]:
        rec = nq[g["idx"]]
        paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
        enc, w = obj.decode_with_special_attention(question=rec["question"], paras=paras, scores=[0.1, 1, 1, 1, 1])
        T = enc["input_ids"].shape[1]
        cb = obj._bias(w, obj.layers_to_be_modified)
        with A.reweighting(obj.model, cb), torch.no_grad():
            out = obj.model.generate(**enc, **obj._generate_kwargs(), output_scores=True, return_dict_in_generate=True)
            last = obj.model(**enc).logits[0, -1].float().cpu()
        d = (last - torch.tensor(g["last_logits"])).abs()
        assert d.max() < 0.15 and d.mean() < 0.03, (d.max().item(), d.mean().item())
        ids = out.sequences[0].tolist()
        gaps = _gaps(out.scores)
        ref = g["ids"]
        assert ids[:T] == ref[:T]
        for t in range(T, min(len(ids), len(ref))):
            if ids[t] != ref[t]:
                assert gaps[t - T] < 0.05 or min(gaps[:t - T + 1]) < 0.05, (t - T, gaps[t - T])
                break
        else:
            assert len(ids) == len(ref)
            prompt, output = obj.run_RAG_with_attention_weighting(question=rec["question"], paras=paras,
                                                                  scores=[0.1, 1, 1, 1, 1])
            assert prompt == g["prompt"] and output == g["output"]


def test_engine_batched_decode_matches_dropin(paths, nq, gpu_device):
    heads = {0: [1], 1: [0, 3], 3: [2]}
    obj = _drop_in(paths, "llama3", heads, gpu_device)
    qs = [nq[i] for i in range(4)]
    args = ([q["question"] for q in qs], [q["ori_fake"] + q["reranked_dense_ctxs"] for q in qs],
            [[0.1, 1, 1, 1, 1]] * 4)
    batched = obj.run_RAG_batch(*args, max_new_tokens=24, use_graph=True)
    eager = obj.run_RAG_batch(*args, max_new_tokens=24, use_graph=False)
    assert batched == eager
    from cram_amd import attention as A
    for i, q in enumerate(qs):
        enc, w = obj.decode_with_special_attention(question=args[0][i], paras=args[1][i], scores=args[2][i])
        cb = obj._bias(w, heads)
        with A.reweighting(obj.model, cb), torch.no_grad():
            out = obj.model.generate(**enc, do_sample=False, max_new_tokens=24, output_scores=True,
                                     return_dict_in_generate=True, eos_token_id=obj._generate_kwargs()["eos_token_id"])
        ref = out.sequences[0, enc["input_ids"].shape[1]:].tolist()
        eng_ids = obj.engine.generate([enc["input_ids"][0]], [w.cpu()], heads, max_new_tokens=24,
                                      eos_ids=obj._generate_kwargs()["eos_token_id"])[0]
        gaps = _gaps(out.scores)
        for t in range(min(len(ref), len(eng_ids))):
            if ref[t] != eng_ids[t]:
                assert min(gaps[:t + 1]) < 0.05, (i, t, gaps[t])
                break


def test_engine_repetition_penalty_matches_dropin(paths, nq, gpu_device):
    """Qwen chat checkpoints ship generation_config.repetition_penalty = 1.05, which model.generate applies in
    greedy decoding: run_RAG_batch (engine, graph-replayed) must apply it too.  The tiny Qwen2's config is set to
    1.05 and to 1.5 (a penalty that changes ids within 24 tokens); ids equal the drop-in's model.generate up to
    the first near-tie (top-2 gap < 0.05 after the penalty)."""
    heads = {0: [0], 2: [1]}
    obj = _drop_in(paths, "qwen2", heads, gpu_device)
    qs = [nq[i] for i in range(3)]
    args = ([q["question"] for q in qs], [q["ori_fake"] + q["reranked_dense_ctxs"] for q in qs],
            [[0.1, 1, 1, 1, 1]] * 3)
    from cram_amd import attention as A
    gc = obj.model.generation_config
    old = gc.repetition_penalty
    try:
        for pen in (1.05, 1.5):
            gc.repetition_penalty = pen
            assert obj._greedy_processors() == pen
            batched = obj.run_RAG_batch(*args, max_new_tokens=24, use_graph=True)
            assert batched == obj.run_RAG_batch(*args, max_new_tokens=24, use_graph=False)
            for i in range(3):
                enc, w = obj.decode_with_special_attention(question=args[0][i], paras=args[1][i], scores=args[2][i])
                cb = obj._bias(w, heads)
                with A.reweighting(obj.model, cb), torch.no_grad():
                    out = obj.model.generate(**enc, do_sample=False, max_new_tokens=24, output_scores=True,
                                             return_dict_in_generate=True)
                ref = out.sequences[0, enc["input_ids"].shape[1]:].tolist()
                got = obj.engine.generate([enc["input_ids"][0]], [w.cpu()], heads, max_new_tokens=24,
                                          eos_ids=[gc.eos_token_id] if isinstance(gc.eos_token_id, int)
                                          else list(gc.eos_token_id or []), repetition_penalty=pen)[0]
                gaps = _gaps(out.scores)
                for t in range(min(len(ref), len(got))):
                    if ref[t] != got[t]:
                        assert min(gaps[:t + 1]) < 0.05, (pen, i, t, gaps[t])
                        break
    finally:
        gc.repetition_penalty = old


def test_batched_sweep_equals_unbatched_on_gpu(fbh, nq):
    from cram_amd import sweep
    from cram_amd.bias import CredibilityBias
    obj = fbh["qwen2"]
    eng = obj.engine
    rec = nq[1]
    enc, w = obj.decode_with_special_attention(question=rec["question"], paras=rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                               scores=[0, 1, 1, 1, 1], answer=rec["wrong_answer"])
    ans = obj.answer_ids(rec["wrong_answer"]).to(gpu := eng.device)
    n = ans.numel()
    L, H = eng.spec.num_layers, eng.spec.num_heads
    ids = enc["input_ids"]

    def s(cb):
        hid = eng.forward_hidden(ids, cb, out_rows=n)[0]
        return eng.answer_logits(hid, ans.to(torch.int32)).sum().item()

    ori = s(None)
    un = np.array([[ori - s(CredibilityBias.build([w.cpu()], {l: [h]}, L, H, gpu)) for h in range(H)] for l in range(L)])
    sw = sweep.ie_question(eng, ids[0], w[0].cpu(), ans.cpu()).double().cpu().numpy()
    assert np.abs(sw - un).max() < 0.05, np.abs(sw - un).max()


@pytest.mark.parametrize("kind", ["llama3", "qwen2", "qwen2_gqa7"])
def test_answer_logprobs_match_reference_hook(paths, nq, gpu_device, kind):
    """G6: re-weighted answer-token log-probabilities through the drop-in (transformers model + cram_hip
    attention) vs the reference hook path.  Bar: per token |ours - fp32 truth| <= 2.5 x the reference's own
    bf16 error on that sample + 0.01 (truth = the reference hook on the float32 copy of the weights)."""
    from cram_amd.re_weighting import Re_Weighting_Strategy
    rows = [r for r in _load(_gold_files(kind)[2]) if r["kind"] == kind]
    truth = {(r["idx"], r["scores"], r["heads"]): np.array(r["logprobs"]) for r in rows if r["fp32"]}
    objs = {}
    worst = 0.0
    agg = parity.Aggregate()
    for r in rows:
        if r["fp32"]:
            continue
        if r["heads"] not in objs:
            objs[r["heads"]] = Re_Weighting_Strategy(model_name=paths[kind],
                                                     layers_to_be_modified=r["layers_to_heads"])
        obj = objs[r["heads"]]
        rec = nq[r["idx"]]
        scores = [0.1, 1, 1, 1, 1] if r["scores"] == "ideal" else [0, 1, 1, 1, 1]
        lp = obj.answer_logprobs(question=rec["question"], paras=rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                 scores=scores, answer=rec["wrong_answer"])
        assert lp.is_cuda and lp.dtype == torch.float32 and lp.numel() == r["n"]
        t = truth[(r["idx"], r["scores"], r["heads"])]
        ref_err = np.abs(np.array(r["logprobs"]) - t).max()
        err = np.abs(lp.cpu().numpy() - t)
        agg.add("logprob_max", err.max(), ref_err, kind=kind, idx=r["idx"], scores=r["scores"], heads=r["heads"])
        worst = max(worst, err.max() / (ref_err + 1e-3))
    print(f"{kind}: worst error / reference bf16 error = {worst:.2f}")
    agg.check()


def test_cal_logits_batch_equals_per_question(fbh, nq):
    obj = fbh["qwen2"]
    recs = nq[:3]
    args = ([r["question"] for r in recs], [r["ori_fake"] + r["reranked_dense_ctxs"] for r in recs],
            [[0, 1, 1, 1, 1]] * 3, [r["wrong_answer"] for r in recs])
    batch = obj.cal_logits_batch(*args)
    assert batch.shape == (3, obj.model_num_hidden_layers, obj.model_num_attention_heads) and batch.is_cuda
    for i, r in enumerate(recs):
        one = obj.cal_logits_tensor(args[0][i], args[1][i], [0, 1, 1, 1, 1], "", args[3][i])
        assert torch.equal(batch[i], one)


def test_gpt2_config1_family_on_gpu(tmp_path_factory, nq, gpu_device):
    """SURVEY §8d config 1 family (GPT-2: MHA, head_dim 64, transformer.h.{l}.attn) through the drop-in on the
    HIP kernels: re-weighted answer log-probs, the IE grid (per-head forwards: the batched engine is Llama /
    Qwen2 only) and a greedy decode, against the oracle's GPT-2 hook adapter (the reference's hook cannot
    run on GPT-2, so this parity is oracle-pinned only).  Same noise-floor bars as the other families."""
    from transformers import AutoModelForCausalLM
    from cram_amd.re_weighting import Find_Best_Heads, Re_Weighting_Strategy
    from oracle import hook_ref
    root = str(tmp_path_factory.mktemp("gpt2"))
    path, path32 = tm.save_model("gpt2", root), tm.save_model("gpt2", root, fp32=True)
    m16 = AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval()
    m32 = AutoModelForCausalLM.from_pretrained(path32, dtype="auto").eval()
    heads = {"0": [1], "2": [0, 3]}
    rw = Re_Weighting_Strategy(model_name=path, layers_to_be_modified=heads)
    agg = parity.Aggregate()
    for rec in nq[:3]:
        paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
        lp = rw.answer_logprobs(question=rec["question"], paras=paras, scores=[0.1, 1, 1, 1, 1],
                                answer=rec["wrong_answer"]).cpu().numpy()
        enc, w = rw.decode_with_special_attention(question=rec["question"], paras=paras, scores=[0.1, 1, 1, 1, 1],
                                                  answer=rec["wrong_answer"])
        ids, lw = enc["input_ids"].cpu(), hook_ref.log_weight(w.cpu())
        hi = {int(k): v for k, v in heads.items()}
        truth = hook_ref.answer_logprobs(m32, ids, lw, hi, lp.size).numpy()
        ref = hook_ref.answer_logprobs(m16, ids, lw, hi, lp.size).numpy()
        agg.add("logprob_max", np.abs(lp - truth).max(), np.abs(ref - truth).max(), kind="gpt2")
    agg.check()
    out = rw.run_RAG_with_attention_weighting(question=nq[0]["question"], paras=nq[0]["ori_fake"][:1], scores=[0.1])
    assert isinstance(out, tuple) and isinstance(out[1], str)

    fbh = Find_Best_Heads(model_name=path)
    rec = nq[0]
    paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
    ie = np.array(fbh.cal_logits(question=rec["question"], paras=paras, scores=[0, 1, 1, 1, 1],
                                 wrong_answer=rec["wrong_answer"]))
    enc, w = fbh.decode_with_special_attention(question=rec["question"], paras=paras, scores=[0, 1, 1, 1, 1],
                                               answer=rec["wrong_answer"])
    ids, lw, ans = enc["input_ids"].cpu(), hook_ref.log_weight(w.cpu()), fbh.answer_ids(rec["wrong_answer"])
    truth = hook_ref.ie_grid(m32, ids, lw, ans)
    h = m16.lm_head.register_forward_hook(lambda mod, a, o: torch.nn.functional.linear(a[0].float(), mod.weight.float()))
    try:
        ref = hook_ref.ie_grid(m16, ids, lw, ans)
    finally:
        h.remove()
    ie_tolerance_check(ie, ref, truth)


def test_engine_multi_token_bad_words_match_dropin(paths, nq, gpu_device):
    """bad_words_ids of any length (re_weighting.py:128-129 hands them to generate; transformers'
    NoBadWordsLogitsProcessor): run_RAG_batch bans them on the device inside the captured step graph.  The list is
    built from the un-banned answers so bans fire (a pair inside the answer, a pair starting at the prompt's last id,
    a triple); graph == eager, and ids equal the drop-in's model.generate(bad_words_ids=...) up to the first near-tie."""
    heads = {0: [1], 1: [0, 3], 3: [2]}
    obj = _drop_in(paths, "llama3", heads, gpu_device)
    qs = [nq[i] for i in range(2)]
    args = ([q["question"] for q in qs], [q["ori_fake"] + q["reranked_dense_ctxs"] for q in qs],
            [[0.1, 1, 1, 1, 1]] * 2)
    enc0, w0 = obj.decode_with_special_attention(question=args[0][0], paras=args[1][0], scores=args[2][0])
    g = obj.engine.generate([enc0["input_ids"][0]], [w0.cpu()], heads, max_new_tokens=16)[0]
    assert len(g) >= 8
    bad = [[g[2], g[3]], [int(enc0["input_ids"][0, -1]), g[0]], [g[4], g[5], g[6]]]
    obj.bad_words_ids = bad
    try:
        batched = obj.run_RAG_batch(*args, max_new_tokens=16, use_graph=True)
        assert batched == obj.run_RAG_batch(*args, max_new_tokens=16, use_graph=False)
        from cram_amd import attention as A
        eos = obj._generate_kwargs()["eos_token_id"]
        for i in range(2):
            enc, w = obj.decode_with_special_attention(question=args[0][i], paras=args[1][i], scores=args[2][i])
            cb = obj._bias(w, heads)
            with A.reweighting(obj.model, cb), torch.no_grad():
                out = obj.model.generate(**enc, do_sample=False, max_new_tokens=16, output_scores=True,
                                         return_dict_in_generate=True, eos_token_id=eos, bad_words_ids=bad)
            ref = out.sequences[0, enc["input_ids"].shape[1]:].tolist()
            got = obj.engine.generate([enc["input_ids"][0]], [w.cpu()], heads, max_new_tokens=16, eos_ids=eos,
                                      bad_words_ids=bad)[0]
            if i == 0:
                assert got[0] != g[0]                        # the prompt-spanning pair fired
            gaps = _gaps(out.scores)
            for t in range(min(len(ref), len(got))):
                if ref[t] != got[t]:
                    assert min(gaps[:t + 1]) < 0.05, (i, t, gaps[t])
                    break
    finally:
        obj.bad_words_ids = []
