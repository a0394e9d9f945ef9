"""Generate the golden vectors by running the REFERENCE hot path itself (build container only).

Imports /root/reference/utils/re_weighting.py unmodified and runs it on CPU on
the tiny deterministic models of tests/tiny_models.py.  Harness shims (the
reference source is untouched):
  * `.to("cuda")` (re_weighting.py:98,111) is redirected to the CPU by wrapping
    torch.Tensor.to and BatchEncoding.to for the duration of the run;
  * model directories are named Llama-3-tiny / Qwen2-tiny so the reference picks
    its Llama-3 / Qwen chat branch (re_weighting.py:65,80);
  * for the "fp32 logits" IE variant an lm_head forward hook recomputes the
    logits as an fp32 product of the bf16 hidden states and bf16 weights (the
    fixture-era fp32 logits; the cal_logits arithmetic itself is unchanged).
Outputs (data only) in tests/golden/:
  spans.json.gz     G1  input ids + fp16 weight vectors from decode_with_special_attention
  masks.npz         G2  edit_attention_mask outputs (prefill / decode / given-mask / head subsets)
  tiny_ie.json.gz   G4  cal_logits IE grids (bf16 logits and fp32 logits) + baseline answer logits
  tiny_ie_f32.json.gz G4' cal_logits on the float32 copy of the same weights (IE ground truth)
  generate.json.gz  G5  run_RAG_with_attention_weighting outputs + greedy ids + hooked last-row logits
  logprobs.json.gz  G6  re-weighted answer-token log-probabilities through the reference hook (bf16 + fp32 copies)
  llama2_*.json.gz  G4/G4'/G5/G6 for the fp16 MHA Llama-2 stand-in (`python gen_golden.py llama2`): the reference's
                    default model family, loaded as fp16 by torch_dtype="auto"; its "bf16" IE variant holds the
                    model-dtype (fp16) logits
  qwen2_gqa7_*.json.gz G4/G4'/G6 for the Qwen2 GQA-7 kind (`python gen_golden.py gqa7`): 7 q-heads per kv head and
                    q/k/v bias as in Qwen2-7B, 4 layers x 14 heads (2 kv heads), 12 NQ questions
"""
import contextlib
import gzip
import json
import os
import sys

sys.dont_write_bytecode = True
os.environ.setdefault("TOKENIZERS_PARALLELISM", "false")

import numpy as np  # noqa: E402
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference/utils")
from tests import tiny_models as tm  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
MODEL_ROOT = "/tmp/cram_golden_models"
torch.set_num_threads(8)


@contextlib.contextmanager
def cuda_to_cpu():
    from transformers.tokenization_utils_base import BatchEncoding
    t_to, b_to = torch.Tensor.to, BatchEncoding.to

    def fix(a, kw):
        a = tuple("cpu" if (isinstance(x, str) and x.startswith("cuda")) else x for x in a)
        if isinstance(kw.get("device"), str) and kw["device"].startswith("cuda"):
            kw["device"] = "cpu"
        return a, kw

    def tensor_to(self, *a, **kw):
        a, kw = fix(a, kw)
        return t_to(self, *a, **kw)

    def batch_to(self, *a, **kw):
        a, kw = fix(a, kw)
        return b_to(self, *a, **kw)

    torch.Tensor.to, BatchEncoding.to = tensor_to, batch_to
    try:
        yield
    finally:
        torch.Tensor.to, BatchEncoding.to = t_to, b_to


def load_data(ds):
    with gzip.open(os.path.join(REPO, "data", f"{ds}_1000.json.gz"), "rt", encoding="utf-8") as f:
        return json.load(f)


def score_variants(rec):
    """(name, paras, scores, answer) per the reference's callers (RAG_test.py:64-107, find_best_heads.py:43-50)."""
    ctx = rec["ori_fake"] + rec["reranked_dense_ctxs"]
    out = [("ideal", ctx, [0.1, 1.0, 1.0, 1.0, 1.0], ""),
           ("sweep", ctx, [0, 1, 1, 1, 1], rec["wrong_answer"])]
    raw = np.array([3, 7, 10, 0, 5])
    sc = (raw - raw.min()) / (raw - raw.min()).max()
    comb = sorted(zip(sc.tolist(), ctx), key=lambda x: x[0])
    out.append(("gpt", [c for _, c in comb], [s for s, _ in comb], ""))
    return out


def gen_spans(rw):
    recs = {"nq": load_data("nq")[:12], "trivia": load_data("trivia")[:4]}
    rows = []
    for kind in ("llama3", "qwen2"):
        path = tm.save_model(kind, MODEL_ROOT)
        obj = object.__new__(rw.Re_Weighting_Strategy)
        from transformers import AutoTokenizer
        obj.tokenizer = AutoTokenizer.from_pretrained(path)
        obj.model_name = path
        for ds, rr in recs.items():
            for i, rec in enumerate(rr):
                for name, paras, scores, answer in score_variants(rec):
                    with cuda_to_cpu():
                        inputs, w = obj.decode_with_special_attention(question=rec["question"], paras=paras,
                                                                      scores=scores, answer=answer)
                    rows.append({"kind": kind, "ds": ds, "idx": i, "variant": name, "paras": paras,
                                 "question": rec["question"], "scores": scores, "answer": answer,
                                 "input_ids": inputs["input_ids"][0].tolist(),
                                 "weight": w[0].float().tolist()})
    with gzip.open(os.path.join(OUT, "spans.json.gz"), "wt", encoding="utf-8") as f:
        json.dump(rows, f)
    print("spans", len(rows))


def gen_masks(rw):
    obj = object.__new__(rw.Re_Weighting_Strategy)
    obj.model_num_attention_heads = 4
    gen = torch.Generator().manual_seed(5)
    W = 24
    w = torch.ones((1, W), dtype=torch.float16)
    w[:, 3:9] = 0.1
    w[:, 9:14] = 0.0
    w[:, 14:18] = 0.5
    lw = torch.log(w)
    out = {"lw": lw.float().numpy()}
    for dt_name, dt in (("bf16", torch.bfloat16), ("fp16", torch.float16), ("fp32", torch.float32)):
        for heads_name, heads in (("h1", [1]), ("hall", [0, 1, 2, 3]), ("h02", [0, 2])):
            T = 30
            kw = {"hidden_states": torch.zeros((1, T, 8), dtype=dt), "attention_mask": None,
                  "position_ids": torch.arange(T)[None]}
            _, kw = obj.edit_attention_mask(None, (), kw, lw, heads)
            out[f"prefill_{dt_name}_{heads_name}"] = kw["attention_mask"].float().numpy()
            kw = {"hidden_states": torch.zeros((1, 1, 8), dtype=dt), "attention_mask": None,
                  "position_ids": torch.tensor([[T + 5]])}
            _, kw = obj.edit_attention_mask(None, (), kw, lw, heads)
            out[f"decode_{dt_name}_{heads_name}"] = kw["attention_mask"].float().numpy()
            given = torch.triu(torch.full((T, T), torch.finfo(dt).min, dtype=dt), 1)[None, None]
            given[..., :, 2] = torch.finfo(dt).min   # a padded key, as transformers would pass it
            kw = {"hidden_states": torch.zeros((1, T, 8), dtype=dt), "attention_mask": given,
                  "position_ids": torch.arange(T)[None]}
            _, kw = obj.edit_attention_mask(None, (), kw, lw, heads)
            out[f"given_{dt_name}_{heads_name}"] = kw["attention_mask"].float().numpy()
    del gen
    np.savez_compressed(os.path.join(OUT, "masks.npz"), **out)
    print("masks", len(out))


def fp32_lm_head(model):
    def hook(mod, args, output):
        return torch.nn.functional.linear(args[0].float(), mod.weight.float())
    return model.lm_head.register_forward_hook(hook)


def gen_ie(rw, kinds=(("llama3", 6), ("qwen2", 8)), out="tiny_ie.json.gz"):
    res = []
    for kind, nq in kinds:
        path = tm.save_model(kind, MODEL_ROOT)
        with cuda_to_cpu():
            fbh = rw.Find_Best_Heads(model_name=path)
        recs = load_data("nq")[:nq]
        for variant in ("bf16", "fp32"):
            h = fp32_lm_head(fbh.model) if variant == "fp32" else None
            for i, rec in enumerate(recs):
                paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
                with cuda_to_cpu():
                    grid = fbh.cal_logits(question=rec["question"], paras=paras, scores=[0, 1, 1, 1, 1],
                                          wrong_answer=rec["wrong_answer"])
                ans = fbh.tokenizer([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
                n = ans.shape[0]
                ori_rows = fbh.ori_logits[0, -n:].float()
                res.append({"kind": kind, "variant": variant, "idx": i, "ie": grid,
                            "answer_ids": ans.tolist(),
                            "ori_answer_logits": ori_rows[torch.arange(n), ans].tolist(),
                            "ori_sum": float(fbh.ori_prob_sum.float())})
                print(kind, variant, i, "ie range", float(np.min(grid)), float(np.max(grid)))
            if h is not None:
                h.remove()
        del fbh
    with gzip.open(os.path.join(OUT, out), "wt", encoding="utf-8") as f:
        json.dump(res, f)


def gen_ie_f32(rw, kinds=(("llama3", 6), ("qwen2", 8)), out="tiny_ie_f32.json.gz"):
    """The reference's cal_logits on the float32 copy of the tiny models: the IE ground truth."""
    res = []
    for kind, nq in kinds:
        path = tm.save_model(kind, MODEL_ROOT, fp32=True)
        with cuda_to_cpu():
            fbh = rw.Find_Best_Heads(model_name=path)
        assert fbh.model.dtype == torch.float32
        for i, rec in enumerate(load_data("nq")[:nq]):
            paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
            with cuda_to_cpu():
                grid = fbh.cal_logits(question=rec["question"], paras=paras, scores=[0, 1, 1, 1, 1],
                                      wrong_answer=rec["wrong_answer"])
            res.append({"kind": kind, "variant": "f32model", "idx": i, "ie": grid})
            print(kind, "f32model", i, float(np.min(grid)), float(np.max(grid)))
        del fbh
    with gzip.open(os.path.join(OUT, out), "wt", encoding="utf-8") as f:
        json.dump(res, f)


def gen_generate(rw, cases=(("llama3", {0: [1], 1: [0, 3], 3: [2]}), ("llama3", {}), ("qwen2", {1: [0]})),
                 out="generate.json.gz"):
    res = []
    recs = load_data("nq")[:4]
    for kind, heads in cases:
        path = tm.save_model(kind, MODEL_ROOT)
        with cuda_to_cpu():
            obj = rw.Re_Weighting_Strategy(model_name=path, layers_to_be_modified=dict(heads), bad_words_ids=[])
        rec_ids = {}
        orig_generate = obj.model.generate

        def generate(**kw):
            lg = obj.model(input_ids=kw["input_ids"], attention_mask=kw["attention_mask"]).logits
            rec_ids["last_logits"] = lg[0, -1].float().tolist()
            out = orig_generate(**kw)
            rec_ids["ids"] = out[0].tolist()
            return out

        obj.model.generate = generate
        for i, rec in enumerate(recs):
            paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
            with cuda_to_cpu():
                prompt, output = obj.run_RAG_with_attention_weighting(question=rec["question"], paras=paras,
                                                                      scores=[0.1, 1, 1, 1, 1])
            res.append({"kind": kind, "heads": {str(k): v for k, v in heads.items()}, "idx": i,
                        "prompt": prompt, "output": output, "ids": rec_ids["ids"],
                        "last_logits": rec_ids["last_logits"]})
            print(kind, heads, i, len(rec_ids["ids"]), repr(output[:60]))
    with gzip.open(os.path.join(OUT, out), "wt", encoding="utf-8") as f:
        json.dump(res, f)


def gen_logprobs(rw, kinds=("llama3", "qwen2"), out="logprobs.json.gz"):
    """Re-weighted teacher-forced answer log-probabilities through the reference's own hook
    (Re_Weighting_Strategy.edit_attention_mask registered exactly as re_weighting.py:119-123 does),
    for the bf16 tiny models and their float32 copies (the ground truth)."""
    from functools import partial
    res = []
    recs = load_data("nq")[:3]
    for kind in kinds:
        for fp32 in (False, True):
            path = tm.save_model(kind, MODEL_ROOT, fp32=fp32)
            with cuda_to_cpu():
                obj = rw.Re_Weighting_Strategy(model_name=path, layers_to_be_modified={}, bad_words_ids=[])
            L, H = obj.model.config.num_hidden_layers, obj.model.config.num_attention_heads
            head_sets = {"sel": {0: [1], 1: [0, H - 1], L - 1: [H - 1]},
                         "all": {l: list(range(H)) for l in range(L)}}
            for i, rec in enumerate(recs):
                paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
                n = obj.tokenizer([rec["wrong_answer"]], return_tensors="pt")["input_ids"].shape[1] - 1
                for sname, scores in (("ideal", [0.1, 1, 1, 1, 1]), ("sweep", [0, 1, 1, 1, 1])):
                    with cuda_to_cpu():
                        mi, aw = obj.decode_with_special_attention(question=rec["question"], paras=paras,
                                                                   scores=scores, answer=rec["wrong_answer"])
                    ids = mi["input_ids"]
                    T = ids.shape[1]
                    for hname, heads in head_sets.items():
                        hooks = []
                        for layer_idx, head_idx in heads.items():
                            module = obj.model.get_submodule(f"model.layers.{layer_idx}.self_attn")
                            hooks.append(module.register_forward_pre_hook(
                                partial(obj.edit_attention_mask, attention_weight=torch.log(aw), head_idx=head_idx),
                                with_kwargs=True))
                        with torch.no_grad(), cuda_to_cpu():
                            lg = obj.model(**mi).logits
                        for hk in hooks:
                            hk.remove()
                        lp = torch.log_softmax(lg[0, T - n - 1:T - 1].float(), dim=-1)
                        lp = lp.gather(1, ids[0, T - n:].view(n, 1)).view(n)
                        res.append({"kind": kind, "fp32": fp32, "idx": i, "scores": sname, "heads": hname,
                                    "layers_to_heads": {str(k): v for k, v in heads.items()}, "n": n,
                                    "ids": ids[0].tolist(), "logprobs": lp.tolist()})
                        print(kind, fp32, i, sname, hname, [round(x, 4) for x in lp.tolist()])
            del obj
    with gzip.open(os.path.join(OUT, out), "wt", encoding="utf-8") as f:
        json.dump(res, f)


def main():
    import re_weighting as rw  # the reference module, unmodified
    which = sys.argv[1:] or ["spans", "masks", "ie", "ie32", "generate", "logprobs"]
    if "spans" in which:
        gen_spans(rw)
    if "masks" in which:
        gen_masks(rw)
    if "ie" in which:
        gen_ie(rw)
    if "ie32" in which:
        gen_ie_f32(rw)
    if "generate" in which:
        gen_generate(rw)
    if "logprobs" in which:
        gen_logprobs(rw)
    if "llama2" in which:
        gen_ie(rw, (("llama2", 3),), "llama2_ie.json.gz")
        gen_ie_f32(rw, (("llama2", 3),), "llama2_ie_f32.json.gz")
        gen_generate(rw, (("llama2", {0: [1], 2: [0, 3]}), ("llama2", {})), "llama2_generate.json.gz")
        gen_logprobs(rw, ("llama2",), "llama2_logprobs.json.gz")
    if "gqa7" in which:
        # Qwen2-7B's GQA-7 grouping with q/k/v bias, 4 layers x 14 heads (56 IE values per question)
        gen_ie(rw, (("qwen2_gqa7", 12),), "qwen2_gqa7_ie.json.gz")
        gen_ie_f32(rw, (("qwen2_gqa7", 12),), "qwen2_gqa7_ie_f32.json.gz")
        gen_logprobs(rw, ("qwen2_gqa7",), "qwen2_gqa7_logprobs.json.gz")


if __name__ == "__main__":
    main()
