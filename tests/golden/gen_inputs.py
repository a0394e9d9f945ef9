"""Rebuild the NQ-1000 / TriviaQA-1000 inputs from the reference's saved prompts.

Runs ONLY in the build container (reads /root/reference).  The reference's
dataset files (nq_1000_bge.json, trivia_1000_bge.json) are absent
(/root/reference/.MISSING_LARGE_BLOBS), but every saved prompt in
results/<ds>/llama3/with_contexts/details/ori_fake_reranked_dense_top4.json is the
raw get_prompt() output (RAG_test.py:126 -> RAG.py:140, prompt.py:4-12) over
contexts = ori_fake[:1] + reranked_dense_ctxs[:4] (RAG_test.py:66-87), so the
passages can be cut back out.  Each rebuilt record is checked by re-rendering
the prompt and requiring byte equality.

Output: data/<ds>_1000.json.gz  [{id, question, ori_fake[1], reranked_dense_ctxs[4],
reference[], wrong_answer}]  (data only, no reference source).
"""
import gzip
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle.hook_ref import get_prompt  # noqa: E402

REF = "/root/reference"
HEAD = "Given the following information: \n"
TAIL = "\nAnswer the following question based on the given information or your internal knowledge"


def split_passages(prompt: str, n: int):
    assert prompt.startswith(HEAD)
    end = prompt.index(TAIL)
    body = prompt[len(HEAD):end]
    assert body.startswith("Passage-0: ")
    cuts = [0]
    pos = 0
    for i in range(1, n):
        pos = body.index(f"\nPassage-{i}: ", pos)
        cuts.append(pos + 1)
    cuts.append(len(body) + 1)
    out = []
    for i in range(n):
        seg = body[cuts[i]:cuts[i + 1] - 1]
        prefix = f"Passage-{i}: "
        assert seg.startswith(prefix)
        out.append(seg[len(prefix):])
    return out


def rebuild(ds: str):
    path = f"{REF}/results/{ds}_1000_bge/llama3/with_contexts/details/ori_fake_reranked_dense_top4.json"
    with open(path, encoding="utf-8") as f:
        rows = json.load(f)
    recs = []
    for r in rows:
        paras = split_passages(r["prompt"], 5)
        assert get_prompt(paras, r["question"], "") == r["prompt"], r["id"]
        recs.append({"id": r["id"], "question": r["question"], "ori_fake": paras[:1],
                     "reranked_dense_ctxs": paras[1:], "reference": r["reference"],
                     "wrong_answer": r["wrong answer"]})
    out = os.path.join(REPO, "data", f"{ds}_1000.json.gz")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with gzip.open(out, "wt", encoding="utf-8", compresslevel=9) as f:
        json.dump(recs, f, ensure_ascii=False)
    print(ds, len(recs), "->", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    for ds in ("nq", "trivia"):
        rebuild(ds)
