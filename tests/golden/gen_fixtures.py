"""Copy the reference's own result fixtures (data only) into tests/golden/ (build container only).

  heads_fixtures.npz     datasets/<ds>/<model>/heads_scores.json ([100, L, H] per-question IE of the
                         real models), heads_scores_mean.json (ranking) and selected_heads.json
                         (top-k) -> the ranking / top-k known-answer tests
  eval_fixtures.json.gz  results*/.../details/*.json rows (LLM_answer, reference, Eval, f1_score) and
                         the *_accuracy summaries -> the EM / F1 known-answer tests
"""
import glob
import gzip
import json
import os

import numpy as np

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, "tests", "golden")

EVAL_FILES = [
    "results_ideal_setting/nq_1000_bge/llama3/with_contexts/details/ori_fake_reranked_dense_top4_weighting_ideal_heads894.json",
    "results_gpt_setting/nq_1000_bge/llama3/with_contexts/details/ori_fake_reranked_dense_top4_weighting_heads894.json",
    "results/nq_1000_bge/llama3/with_contexts/details/ori_fake_reranked_dense_top4.json",
    "results_ideal_setting/nq_1000_bge/qwen/with_contexts/details/ori_fake_reranked_dense_top4_weighting_ideal_heads789.json",
    "results/nq_1000_bge/llama3/without_contexts/details/no_contexts.json",
]


def heads():
    arrs = {}
    for d in sorted(glob.glob(f"{REF}/datasets/*/*")):
        ds, model = d.split("/")[-2:]
        key = f"{ds}__{model}"
        p = os.path.join(d, "heads_scores.json")
        if os.path.exists(p):
            with open(p) as f:
                arrs[key + "__scores"] = np.asarray(json.load(f), dtype=np.float64)
        with open(os.path.join(d, "heads_scores_mean.json")) as f:
            mean = json.load(f)
        arrs[key + "__mean_values"] = np.asarray([m[0] for m in mean], dtype=np.float64)
        arrs[key + "__mean_lh"] = np.asarray([m[1] for m in mean], dtype=np.int32)
        with open(os.path.join(d, "selected_heads.json")) as f:
            sel = json.load(f)
        k = sum(len(v) for v in sel.values())
        flat = [(int(l), int(h)) for l, hs in sel.items() for h in hs]
        arrs[key + "__selected"] = np.asarray(flat, dtype=np.int32).reshape(-1, 2)
        arrs[key + "__selected_k"] = np.asarray([k], dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "heads_fixtures.npz"), **arrs)
    print("heads", sorted(arrs))


def evals():
    out = []
    for rel in EVAL_FILES:
        with open(os.path.join(REF, rel), encoding="utf-8") as f:
            rows = json.load(f)
        acc_path = os.path.join(REF, rel).replace(".json", "_accuracy").replace("/details", "")
        with open(acc_path, encoding="utf-8") as f:
            acc = f.read()
        out.append({"file": rel, "accuracy": acc,
                    "rows": [{k: r[k] for k in ("LLM_answer", "reference", "Eval", "f1_score")} for r in rows]})
    with gzip.open(os.path.join(OUT, "eval_fixtures.json.gz"), "wt", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False)
    print("eval", len(out))


if __name__ == "__main__":
    heads()
    evals()
