"""ORACLE — test infrastructure only (never the product path).

A CPU restatement of the reference's credibility re-weighting hot path
(/root/reference/utils/re_weighting.py, utils/prompt.py, utils/find_best_heads.py).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker / the timed CPU baseline.  The
``cram_amd`` package never imports it.

Pinning: the restatement is checked against golden vectors that
``tests/golden/gen_golden.py`` produced by importing and running the reference
itself in the build container (spans, hook masks, tiny-model logits, IE grids,
greedy outputs) and against the reference's own fixtures
(datasets/*/*/heads_scores*.json, selected_heads.json, results*/details).
"""
