"""Where does the tiny models' IE error come from?  (the Qwen2 outliers.)

Test tooling (imports the oracle as a checker).  For every golden question of a tiny kind, the IE grid of
Find_Best_Heads.cal_logits (re_weighting.py:152-175) is computed several ways, each compared with the float32 truth
(the reference run on the float32 copy of the same weights, tests/golden/*_f32.json.gz):
  sweep          the product: head-batched layer-suffix sweep on the HIP kernels (fused GEMM epilogues)
  sweep_lib      the same sweep with every projection on hipBLASLt + the separate RoPE / SiLU-mul / residual passes
  per_head_hip   the reference ALGORITHM (one hooked forward per unit) on transformers + the cram_hip kernels
  ref_gpu_sdpa   the reference algorithm on transformers' own GPU kernels (sdpa, dense-mask hook), bf16
  ref_gpu_eager  the same with transformers' eager attention
  ref_cpu_eager  the same on the host CPU, eager attention
  golden         the reference itself as the fixture holds it (CPU, sdpa)
Every IE uses fp32 answer logits (the fixture-era convention of tests/golden 'fp32').  One JSON line per (kind,
question, arm) with mean / max |IE - truth|, then per-arm aggregates over the informative questions (not 0/0) and
over the original three Qwen2 questions, as ratios to the golden reference's own error.

  python tools/ie_noise_probe.py --kinds qwen2 qwen2_gqa7 llama3 --out gpurun_out/ie_noise.jsonl
"""
import argparse
import gzip
import json
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tests import tiny_models as tm  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")
FILES = {"qwen2_gqa7": ("qwen2_gqa7_ie.json.gz", "qwen2_gqa7_ie_f32.json.gz")}


def load(name):
    with gzip.open(os.path.join(GOLD, name), "rt", encoding="utf-8") as f:
        return json.load(f)


def fp32_lm_head(model):
    return model.lm_head.register_forward_hook(
        lambda mod, a, o: torch.nn.functional.linear(a[0].float(), mod.weight.float()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", nargs="+", default=["qwen2", "qwen2_gqa7", "llama3"])
    ap.add_argument("--out", default="gpurun_out/ie_noise.jsonl")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    from transformers import AutoModelForCausalLM
    from cram_amd import engine as E
    from cram_amd.re_weighting import Find_Best_Heads
    from oracle import hook_ref
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    with gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt") as f:
        nq = json.load(f)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    out = open(args.out, "w")
    root = tempfile.mkdtemp(prefix="ie_noise_")
    summary = {}
    for kind in args.kinds:
        f_ie, f_t = FILES.get(kind, ("tiny_ie.json.gz", "tiny_ie_f32.json.gz"))
        gold = [x for x in load(f_ie) if x["kind"] == kind and x["variant"] == "fp32"]
        truth = {x["idx"]: np.array(x["ie"]) for x in load(f_t) if x["kind"] == kind}
        path = tm.save_model(kind, root)
        fbh = Find_Best_Heads(model_name=path)
        dev = fbh.device
        ref_models = {}
        for impl in ("sdpa", "eager"):
            m = AutoModelForCausalLM.from_pretrained(path, dtype=torch.bfloat16, attn_implementation=impl).eval()
            ref_models[("gpu", impl)] = m.to(dev)
        if not args.no_cpu:
            ref_models[("cpu", "eager")] = AutoModelForCausalLM.from_pretrained(
                path, dtype=torch.bfloat16, attn_implementation="eager").eval()
        for g in gold:
            i = g["idx"]
            rec = nq[i]
            paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
            if fbh.answer_ids(rec["wrong_answer"]).numel() == 0:      # one-token answer: IE == 0 in every run
                continue
            kw = dict(question=rec["question"], paras=paras, scores=[0, 1, 1, 1, 1], wrong_answer=rec["wrong_answer"])
            grids = {"golden": np.array(g["ie"])}
            grids["sweep"] = fbh.cal_logits_tensor(**kw).double().cpu().numpy()
            saved = E.FUSED_MLP, E.FUSED_QKV, E.FUSED_RESIDUAL
            E.FUSED_MLP = E.FUSED_QKV = E.FUSED_RESIDUAL = False
            try:
                grids["sweep_lib"] = fbh.cal_logits_tensor(**kw).double().cpu().numpy()
            finally:
                E.FUSED_MLP, E.FUSED_QKV, E.FUSED_RESIDUAL = saved
            enc, w = fbh.decode_with_special_attention(question=rec["question"], paras=paras, scores=[0, 1, 1, 1, 1],
                                                       answer=rec["wrong_answer"])
            ans = fbh.answer_ids(rec["wrong_answer"])
            grids["per_head_hip"] = fbh._ie_per_head(enc["input_ids"], w, ans, False,
                                                     list(range(fbh.model_num_hidden_layers))).double().cpu().numpy()
            lw = hook_ref.log_weight(w.cpu())
            for (where, impl), m in ref_models.items():
                h = fp32_lm_head(m)
                try:
                    d = dev if where == "gpu" else torch.device("cpu")
                    grids[f"ref_{where}_{impl}"] = hook_ref.ie_grid(m, enc["input_ids"].to(d), lw.to(d), ans.to(d))
                finally:
                    h.remove()
            t = truth[i]
            for arm, gr in grids.items():
                e = np.abs(gr - t)
                rec_o = {"kind": kind, "idx": i, "arm": arm, "mean": float(e.mean()), "max": float(e.max()),
                         "informative": bool(np.abs(grids["golden"] - t).max() > 0 or e.max() > 0)}
                out.write(json.dumps(rec_o) + "\n")
                out.flush()
                if rec_o["informative"]:
                    for sub in ("all", "first3") if (kind == "qwen2" and i < 3) else ("all",):
                        s = summary.setdefault((kind, sub, arm), [0.0, 0.0, 0])
                        s[0] += rec_o["mean"]
                        s[1] += rec_o["max"]
                        s[2] += 1
            print(kind, i, {a: round(float(np.abs(gr - t).max()), 4) for a, gr in grids.items()}, flush=True)
        del fbh, ref_models
        torch.cuda.empty_cache()
    for (kind, sub, arm), (sm, sx, n) in sorted(summary.items()):
        gm, gx, _ = summary[(kind, sub, "golden")]
        line = {"kind": kind, "subset": sub, "arm": arm, "n": n, "mean_ratio_to_golden": sm / max(gm, 1e-12),
                "max_ratio_to_golden": sx / max(gx, 1e-12), "sum_mean": sm, "sum_max": sx}
        out.write(json.dumps({"aggregate": line}) + "\n")
        print(json.dumps(line), flush=True)
    out.close()


if __name__ == "__main__":
    main()
