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
    """The row-exact sweep (the default since round 6) drops the per-layer un-perturbed variant (sweep.py) because an un-perturbed row
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
    sweep.ROW_EXACT = True                          # the default mode (CRAM_SWEEP_ROW_EXACT=0 turns it off)
    try:
        _row_exact_checks(eng, ids, w16, ans, sweep, CredibilityBias)
    finally:
        sweep.ROW_EXACT = prev


def test_grouped_batches_are_bit_identical(setup):
    """sweep.group_variants at the Llama-3-8B shape: consecutive swept layers in one growing batch (each joining
    after its own attention) give the IE grid one batch per layer gives, bit for bit in the row-exact mode -- the
    4-wave GEMM rounds a row the same whatever M and the row's place, attention and RMSNorm are per sequence / row."""
    from cram_amd import sweep
    eng, ids, w16, ans = setup
    layers = [0, 1, 2, 3, 4, 5, 28, 29, 30, 31]
    prev = sweep.SWEEP_GROUP
    try:
        sweep.SWEEP_GROUP = 1
        a = sweep.ie_question(eng, ids, w16, ans, layers=layers)
        for g in (3, 4):
            sweep.SWEEP_GROUP = g
            b = sweep.ie_question(eng, ids, w16, ans, layers=layers)
            assert sweep.row_exact(eng)
            assert torch.equal(a, b), (g, (a - b).abs().max().item())
    finally:
        sweep.SWEEP_GROUP = prev


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


GRIDS = os.path.join(REPO, "tests", "golden", "fullsize_grids_llama3_8b.npz")
# per-question standard deviation of the top-k overlap difference (one valid bf16 rounding's overlap with the float32
# truth minus another's) at the k the bar checks: pooled over (row-exact - reference hook) and (default - reference
# hook) on the 13 full grids of round 5 (profiles/r05/rowexact/grid_q*.txt; tools/fullsize_grids.py regenerates them)
SIGMA_K = {894: 16.6, 506: 15.5, 100: 18.2, 10: 1.42}


def _weights_checksum(eng):
    parts = []
    for lw in eng.layers:
        for t in (lw.wqkv, lw.wo, lw.wgu, lw.wd):
            parts.append(float(t[::97, ::89].double().sum()))
    parts.append(float(eng.embed[::997, ::13].double().sum()))
    parts.append(float(eng.lm_head[::997, ::13].double().sum()))
    return parts


def _question(eng, qi):
    from transformers import AutoTokenizer
    from cram_amd import spans
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3"))
    data = json.load(gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8"))
    rec = data[qi]
    _, enc, w, _ = spans.encode(tok, "Meta-Llama-3-8B-Instruct", rec["question"],
                                rec["ori_fake"] + rec["reranked_dense_ctxs"], [0, 1, 1, 1, 1], rec["wrong_answer"])
    ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
    return enc["input_ids"][0].to(eng.device), w[0], ans.to(eng.device)


def test_full_grid_fixture_reproduces(setup):
    """The cached full grids of the multi-question bar (tests/golden/fullsize_grids_llama3_8b.npz, written by
    tools/fullsize_grids.py on this image) are what the reference algorithm and the float32 truth give on THIS
    engine: the weights' checksum matches, and one question's grids recomputed live (the reference algorithm in bf16:
    transformers + the dense-mask hook, oracle/hook_ref.py; the float32 truth, tests/fp32_llama.py) equal them."""
    import numpy as np
    from oracle import cpu_baseline, hook_ref
    from tests.fp32_llama import Fp32Llama
    eng = setup[0]
    fx = np.load(GRIDS)
    assert np.allclose(_weights_checksum(eng), fx["checksum"], rtol=0, atol=1e-9), "engine differs from the fixture's"
    i = int(np.nonzero(fx["qi"] == 3)[0][0])
    ids, w16, ans = _question(eng, 3)
    assert ids.numel() == int(fx["T"][i])
    hf = cpu_baseline.hf_model_from_engine(eng).to(eng.device)
    hook = hook_ref.ie_grid(hf, ids[None], hook_ref.log_weight(w16.view(1, -1)).to(eng.device), ans, upcast_logits=True)
    del hf
    torch.cuda.empty_cache()
    f32 = Fp32Llama(eng)
    truth = f32.ie_grid(ids, torch.log(w16.to(eng.device).float()), ans).numpy()
    del f32
    torch.cuda.empty_cache()
    dt, dh = float(np.abs(truth - fx["truth"][i]).max()), float(np.abs(hook - fx["hook"][i]).max())
    print(f"\nq3 live vs cached: truth max |diff| {dt:.2e}, reference hook max |diff| {dh:.2e}")
    assert dt < 2e-3 and dh < 2e-2, (dt, dh)


def test_full_grid_topk_sets_at_the_path_k(setup):
    """The north star's "identical top-k head set" at the k the path uses (894 nq/llama3, 506 trivia/llama3,
    selected_heads.json; RAG_test.py:50-58) over the full 32 x 32 grids of several NQ questions: ours (the sweep, live),
    the reference algorithm in bf16 and the float32 truth (cached: test_full_grid_fixture_reproduces), each ranked as
    find_best_heads.py:113-150 ranks (fixed tie-break).  With random-init weights the IE signal (|IE| ~ 0.02) is below
    every bf16 run's noise, so the overlap of a top-k set with the truth's is a noisy statistic of the rounding; the
    bars are therefore over the questions:
      * accuracy: our RMS error against the truth over every unit of every question <= the reference algorithm's own;
      * overlap: the mean over questions of (our overlap - the reference's) >= -3 sigma_k / sqrt(Nq), sigma_k the
        measured per-question spread of that difference between two valid bf16 roundings (SIGMA_K);
      * rank correlation over the grid (mean Spearman vs the truth) within 3 sqrt(2) / sqrt(Nq) of its spread;
      * identity with the truth wherever a question's truth boundary gap exceeds twice our max error there.
    Both sweep modes are measured (the default and the other, sweep.ROW_EXACT); the bars are asserted on the product's
    default and logged for both (profiles/r06/).  The real identity bar, on a model whose IE has signal, is
    tests/test_topk_identity_gpu.py (planted heads)."""
    import math

    import numpy as np
    from cram_amd import heads as Hd
    from cram_amd import sweep

    eng = setup[0]
    fx = np.load(GRIDS)
    assert np.allclose(_weights_checksum(eng), fx["checksum"], rtol=0, atol=1e-9), "engine differs from the fixture's"
    topk = lambda g, k: {lh for _, lh in Hd.rank_heads(g)[:k]}
    rho = lambda g, t: _spearman(torch.from_numpy(np.ascontiguousarray(g.reshape(-1))),
                                 torch.from_numpy(np.ascontiguousarray(t.reshape(-1))))
    default = sweep.ROW_EXACT
    stats = {m: {"se": 0.0, "n": 0, "ov": {k: [] for k in SIGMA_K}, "rho": [], "ident": []} for m in (default, not default)}
    ref = {"se": 0.0, "n": 0, "ov": {k: [] for k in SIGMA_K}, "rho": []}
    nq = len(fx["qi"])
    try:
        for i, qi in enumerate(fx["qi"].tolist()):
            ids, w16, ans = _question(eng, qi)
            truth, hook = fx["truth"][i].astype(np.float64)[None], fx["hook"][i].astype(np.float64)[None]
            ref["se"] += float(((hook - truth) ** 2).sum())
            ref["n"] += truth.size
            ref["rho"].append(rho(hook, truth))
            for k in SIGMA_K:
                ref["ov"][k].append(len(topk(hook, k) & topk(truth, k)))
            st = np.sort(truth.reshape(-1))[::-1]
            line = [f"q{qi}"]
            for mode in (default, not default):
                sweep.ROW_EXACT = mode
                ours = sweep.ie_question(eng, ids, w16, ans).double().cpu().numpy()[None]
                s = stats[mode]
                s["se"] += float(((ours - truth) ** 2).sum())
                s["n"] += truth.size
                s["rho"].append(rho(ours, truth))
                noise = float(np.abs(ours - truth).max())
                for k in SIGMA_K:
                    s["ov"][k].append(len(topk(ours, k) & topk(truth, k)))
                    if float(st[k - 1] - st[k]) > 2 * noise:
                        s["ident"].append((qi, k, topk(ours, k) == topk(truth, k)))
                line.append(f"{'row-exact' if mode else 'default'}: rms {math.sqrt(((ours - truth) ** 2).mean()):.4f} "
                            + " ".join(f"k={k} {s['ov'][k][-1]}" for k in SIGMA_K))
            line.append(f"reference: rms {math.sqrt(((hook - truth) ** 2).mean()):.4f} "
                        + " ".join(f"k={k} {ref['ov'][k][-1]}" for k in SIGMA_K))
            print(" | ".join(line), flush=True)
    finally:
        sweep.ROW_EXACT = default
    rms_r = math.sqrt(ref["se"] / ref["n"])
    rho_sd = float(np.std(np.array(ref["rho"]), ddof=1)) if nq > 1 else 0.05
    fails = {}
    for mode, s in stats.items():
        name = "row-exact" if mode else "default"
        rms_o = math.sqrt(s["se"] / s["n"])
        f = []
        if rms_o > rms_r:
            f.append(("rms", rms_o, rms_r))
        for k, sig in SIGMA_K.items():
            d = float(np.mean(np.array(s["ov"][k]) - np.array(ref["ov"][k])))
            bar = -3.0 * sig / math.sqrt(nq)
            print(f"{name} k={k}: mean overlap with truth ours {np.mean(s['ov'][k]):.1f} reference "
                  f"{np.mean(ref['ov'][k]):.1f} (difference {d:+.2f}, bar {bar:.2f} over {nq} questions)")
            if d < bar:
                f.append(("overlap", k, d, bar))
        dr = float(np.mean(s["rho"]) - np.mean(ref["rho"]))
        rbar = -3.0 * math.sqrt(2.0) * max(rho_sd, 0.01) / math.sqrt(nq)
        print(f"{name}: rms {rms_o:.5f} vs reference {rms_r:.5f} (ratio {rms_o / rms_r:.3f}, bar 1.0); "
              f"spearman {np.mean(s['rho']):.4f} vs {np.mean(ref['rho']):.4f} (bar {rbar:+.4f}); "
              f"identity checks {len(s['ident'])}, failed {[x for x in s['ident'] if not x[2]]}")
        if dr < rbar:
            f.append(("spearman", dr, rbar))
        f += [("identity",) + x[:2] for x in s["ident"] if not x[2]]
        fails[name] = f
    assert not fails["row-exact" if default else "default"], fails


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
