"""Recover the GPT-setting truthful scores for NQ-1000 and pin the score pipeline (RAG_test.py:64-121).

Runs ONLY in the build container (reads /root/reference result files as data).

1. results_gpt_setting/nq_1000_bge/llama2_13b_chat/with_contexts_score/details/with_contexts_score.json
   holds, per question, every passage followed by "Truthful socre: N" (prompt.py:17).  Each of the five
   rebuilt contexts (data/nq_1000.json.gz) is located in that prompt and its N read back; the ints are
   stored as ori_fake_truthful_scores / reranked_dense_ctxs_truthful_scores (the dataset fields
   RAG_test.py:78,88 read).  A passage text that occurs twice in one question gets its occurrences'
   scores in prompt order (the two assignments render the same prompt).
2. Fixtures from the reference's saved prompts, as original-context indices per question:
   - weighting order: results_gpt_setting/nq_1000_bge/llama2_13b_chat/with_contexts/details/
     ori_fake_reranked_dense_top4_weighting.json (raw get_prompt of the re-ordered contexts);
   - delete kept set: results_gpt_setting/nq_1000_bge/llama3/with_contexts/details/
     ori_fake_reranked_dense_top4_delete.json (raw get_prompt of the kept contexts).
   Both prompts are re-rendered from the indices and required to be byte-equal before writing.
Trivia-1000 has no score prompt in the reference's results, so its truthful scores stay unrecovered.

Output: data/nq_1000.json.gz (two fields added), tests/golden/score_pipeline.json.gz.
"""
import gzip
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle.hook_ref import get_prompt  # noqa: E402

GPT = "/root/reference/results_gpt_setting/nq_1000_bge"


def recover_scores(recs):
    with open(f"{GPT}/llama2_13b_chat/with_contexts_score/details/with_contexts_score.json", encoding="utf-8") as f:
        rows = {r["id"]: r for r in json.load(f)}
    for rec in recs:
        p = rows[rec["id"]]["prompt"]
        ctx = rec["ori_fake"] + rec["reranked_dense_ctxs"]
        used = {}
        out = []
        for c in ctx:
            ms = list(re.finditer(r"Passage-(\d+): " + re.escape(c) + r"Truthful socre: (\d+)\n", p))
            k = used.get(c, 0)
            assert len(ms) > k, (rec["id"], c[:40])
            used[c] = k + 1
            out.append(int(ms[k].group(2)))
        rec["ori_fake_truthful_scores"] = out[:1]
        rec["reranked_dense_ctxs_truthful_scores"] = out[1:]


def prompt_indices(prompt, ctx):
    """Original-context index of each passage of a raw get_prompt() output, in prompt order
    (equal passage texts map to their lowest unused index)."""
    tail = prompt.index("\nAnswer the following question")
    taken, idx, pos, k = set(), [], 0, 0
    while 0 <= prompt.find(f"Passage-{k}: ", pos) < tail:
        pos = prompt.index(f"Passage-{k}: ", pos) + len(f"Passage-{k}: ")
        cand = [i for i, c in enumerate(ctx) if i not in taken and prompt.startswith(c + "\n", pos)]
        assert cand, k
        i = min(cand, key=lambda j: (-len(ctx[j]), j))
        taken.add(i)
        idx.append(i)
        pos += len(ctx[i])
        k += 1
    return idx


def fixtures(recs):
    with open(f"{GPT}/llama2_13b_chat/with_contexts/details/ori_fake_reranked_dense_top4_weighting.json",
              encoding="utf-8") as f:
        wrows = {r["id"]: r for r in json.load(f)}
    with open(f"{GPT}/llama3/with_contexts/details/ori_fake_reranked_dense_top4_delete.json", encoding="utf-8") as f:
        drows = {r["id"]: r for r in json.load(f)}
    out = []
    for rec in recs:
        ctx = rec["ori_fake"] + rec["reranked_dense_ctxs"]
        w = wrows[rec["id"]]["prompt"]
        wi = prompt_indices(w, ctx)
        assert get_prompt([ctx[i] for i in wi], rec["question"], "") == w, rec["id"]
        d = drows[rec["id"]]["prompt"]
        di = prompt_indices(d, ctx)
        assert get_prompt([ctx[i] for i in di], rec["question"], "") == d, rec["id"]
        out.append({"id": rec["id"], "weighting_order": wi, "delete_kept": di})
    return out


def main():
    path = os.path.join(REPO, "data", "nq_1000.json.gz")
    with gzip.open(path, "rt", encoding="utf-8") as f:
        recs = json.load(f)
    recover_scores(recs)
    fx = fixtures(recs)
    with gzip.open(path, "wt", encoding="utf-8", compresslevel=9) as f:
        json.dump(recs, f, ensure_ascii=False)
    out = os.path.join(REPO, "tests", "golden", "score_pipeline.json.gz")
    with gzip.open(out, "wt", encoding="utf-8", compresslevel=9) as f:
        json.dump(fx, f)
    print("nq scores recovered for", len(recs), "questions ->", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
