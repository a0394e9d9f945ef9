"""The noise-floor parity bars of the float-valued outputs, written once.

Every bar compares our error against the float32 truth (the reference hook on the float32 copy of the same weights)
with the reference algorithm's own 16-bit error on the same sample:  ours <= F * reference + A.
  ie_mean / ie_max   the IE grid of cal_logits (re_weighting.py:152-175): mean / max over the grid of |IE - truth|
  logprob_max        the re-weighted answer-token log-probabilities (the hooked forward of re_weighting.py:118-127):
                     max over the answer tokens of |log p - truth|
Achieved ratios (ours / reference) are appended, one JSON line per check, to the file CRAM_PARITY_LOG names (the
suites' evidence run: profiles/r05/parity_ratios.json summarises it); F and A below come from that evidence.
"""
import json
import os

# (F, A) per family
BARS = {"ie_mean": (2.5, 0.01), "ie_max": (2.5, 0.05), "logprob_max": (2.5, 0.01)}


def record(family: str, ours: float, ref: float, **extra) -> None:
    path = os.environ.get("CRAM_PARITY_LOG")
    if not path:
        return
    rec = {"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], "family": family, "ours": float(ours),
           "reference": float(ref), "ratio": float(ours) / max(float(ref), 1e-12)}
    rec.update(extra)
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")


def check(family: str, ours: float, ref: float, **extra) -> None:
    """Record, then assert ours <= F * ref + A for the family."""
    record(family, ours, ref, **extra)
    F, A = BARS[family]
    assert ours <= F * ref + A, (family, float(ours), float(ref), F, A, extra)


def ie_errors(e_ie, e_ref, **extra) -> None:
    """Mean and max |IE - truth| of a grid against the reference's."""
    check("ie_mean", float(e_ie.mean()), float(e_ref.mean()), **extra)
    check("ie_max", float(e_ie.max()), float(e_ref.max()), **extra)
