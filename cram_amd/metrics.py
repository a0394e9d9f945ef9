"""Answer-quality metrics of the reference (eval.py:13-94): SQuAD normalisation, EM, token F1.

These turn decode outputs into the published EM/F1 numbers.
"""
from __future__ import annotations

import json
import re
import string
import unicodedata
from collections import Counter
from typing import List

_PUNCT = set(string.punctuation)
_ARTICLES = re.compile(r"\b(a|an|the)\b")


def normalize_text(s: str) -> str:
    """eval.py:13-29 (NFD, lower, strip punctuation, drop articles, squeeze whitespace)."""
    s = unicodedata.normalize("NFD", s).lower()
    s = "".join(ch for ch in s if ch not in _PUNCT)
    s = _ARTICLES.sub(" ", s)
    return " ".join(s.split())


def f1_score(prediction: str, ground_truth: str) -> float:
    """eval.py:32-51."""
    p = normalize_text(prediction).split()
    g = normalize_text(ground_truth).split()
    if len(p) == 0 and len(g) == 0:
        return 1
    same = sum((Counter(p) & Counter(g)).values())
    if same == 0:
        return 0
    prec, rec = same / len(p), same / len(g)
    return (2 * prec * rec) / (prec + rec)


def exact_match(answer: str, references: List[str]) -> bool:
    """eval.py:54-62."""
    if answer == "":
        return False
    a = normalize_text(answer)
    return any(normalize_text(r) == a for r in references)


def f1_max(prediction: str, answers: List[str]) -> float:
    """eval.py:65-68."""
    return max(f1_score(prediction, a) for a in answers)


def evaluate(rows: list) -> dict:
    """eval.py:71-94 without the file I/O: fills Eval / f1_score per row, returns the summary."""
    cnt, f1s = 0, []
    for d in rows:
        ok = exact_match(d["LLM_answer"], d["reference"])
        d["Eval"] = "Correct" if ok else "Wrong"
        cnt += int(ok)
        d["f1_score"] = f1_max(d["LLM_answer"], d["reference"])
        f1s.append(d["f1_score"])
    n = len(rows)
    return {"accuracy": cnt / n if n else 0.0, "em": cnt, "n": n, "f1": sum(f1s) / n if n else 0.0}


def evaluate_file(path: str) -> dict:
    with open(path, encoding="utf-8") as f:
        rows = json.load(f)
    summary = evaluate(rows)
    with open(path, "w", encoding="utf-8") as f:
        json.dump(rows, f, ensure_ascii=False, indent=4)
    with open(path.replace(".json", "_accuracy").replace("/details", ""), "w", encoding="utf-8") as f:
        f.write(f"Accuracy: {summary['accuracy']:.4f}\n")
        f.write(f"EM: {summary['em']}/{summary['n']}\n")
        f.write(f"F1: {summary['f1']:.4f}\n")
    return summary
