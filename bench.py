"""Benchmark: questions/sec reweighted-decode + heads/sec IE-sweep, Llama-3-8B NQ-1000 (BASELINE.json).

One step = the full Find_Best_Heads IE sweep (32 layers x 32 heads) of ONE NQ
question per GPU (weak scaling; questions are dealt to ranks, no data-path
collective), plus one RCCL all-gather of the IE grids at the end of the timed
region.  The primary `value` is heads/s over all ranks; the batched
reweighted decode (questions/s) is reported next to it as `decode`.

Run:  python bench.py [--gpus N] [--steps K] [--warmup W]
      (N > 1 under `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`)
Weights are random-init of the Llama-3-8B architecture (no checkpoint offline);
prompts are the rebuilt NQ-1000 inputs through the offline BPE tokenizer with
the Llama-3 chat template (mean ~905 tokens with the wrong answer appended).
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "questions/sec reweighted-decode + heads/sec IE-sweep, Llama-3-8B NQ-1000"
PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip table)
PEAK_HBM_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b", choices=["llama3-8b", "qwen2-7b"])
    ap.add_argument("--decode-batch", type=int, default=64)
    ap.add_argument("--decode-tokens", type=int, default=16)
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-units", type=int, default=2)
    ap.add_argument("--blas", default="hipblaslt", choices=["hipblas", "hipblaslt"])
    args = ap.parse_args()

    import torch
    from cram_amd import dist as cdist
    from cram_amd import ops, spans, sweep
    from cram_amd.engine import CrAMEngine, ModelSpec

    rank, world, local = cdist.init()
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from cram_amd import build as _b
    if rank == 0 and _b.needs_build():
        _b.build()
    if world > 1:
        torch.distributed.barrier()

    from cram_amd.engine import configure_blas
    configure_blas(args.blas)
    spec = ModelSpec.llama3_8b() if args.model == "llama3-8b" else ModelSpec.qwen2_7b()
    t0 = time.time()
    eng = CrAMEngine.random(spec, dev, seed=1234, rope_theta=500000.0 if args.model == "llama3-8b" else 1e6)
    torch.cuda.synchronize()
    log(f"[rank {rank}] random-init {args.model} in {time.time() - t0:.1f}s")

    from transformers import AutoTokenizer
    tok = AutoTokenizer.from_pretrained(os.path.join(REPO, "data", "tok_llama3" if args.model == "llama3-8b"
                                                      else "tok_qwen"))
    name = "Meta-Llama-3-8B-Instruct" if args.model == "llama3-8b" else "Qwen2-7B-Instruct"
    with gzip.open(os.path.join(REPO, "data", "nq_1000.json.gz"), "rt", encoding="utf-8") as f:
        nq = json.load(f)

    n_q = (args.warmup + args.steps) * world
    qids = [(s * world + rank) % len(nq) for s in range(args.warmup + args.steps)]
    work = []
    for qi in qids:
        rec = nq[qi]
        paras = rec["ori_fake"] + rec["reranked_dense_ctxs"]
        _, enc, w, _ = spans.encode(tok, name, rec["question"], paras, [0, 1, 1, 1, 1], rec["wrong_answer"])
        ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
        work.append((qi, enc["input_ids"][0].to(dev), w[0], ans.to(dev)))
    torch.cuda.synchronize()
    L, H = spec.num_layers, spec.num_heads

    # ---------------- IE sweep: warmup, then K timed steps (inputs resident in HBM)
    results = []
    for s in range(args.warmup):
        qi, ids, w, ans = work[s]
        results.append(sweep.ie_question(eng, ids, w, ans))
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup step {s} done")
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    ops.TIMER.reset()
    ops.TIMER.enabled = True
    t_start = time.perf_counter()
    flops = 0.0
    timed = []
    for s in range(args.steps):
        qi, ids, w, ans = work[args.warmup + s]
        timed.append(sweep.ie_question(eng, ids, w, ans))
        flops += sweep.sweep_flops(spec, ids.numel(), ans.numel())
        if rank == 0:
            log(f"[rank 0] step {s} enqueued ({time.perf_counter() - t_start:.1f}s)")
    local_ie = torch.stack(timed)
    local_ids = torch.tensor([(args.warmup + s) * world + rank for s in range(args.steps)], dtype=torch.int64)
    full = cdist.gather_rows(local_ie, local_ids, n_q)          # the sweep's RCCL all-gather
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t_start
    ops.TIMER.enabled = False
    kt = ops.TIMER.summary().get("cram_prefill", None)
    el = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    fl = torch.tensor([flops], device=dev, dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(fl)
    elapsed, flops_all = float(el.item()), float(fl.item())
    units = world * args.steps * L * H
    heads_per_s = units / elapsed
    assert torch.isfinite(full[args.warmup * world:]).all(), "non-finite IE"
    mean_T = sum(x[1].numel() for x in work) / len(work)
    log(f"[rank {rank}] IE sweep: {units} units in {elapsed:.2f}s -> {heads_per_s:.1f} heads/s")

    # ---------------- batched reweighted decode (replicas; questions/s), outside the IE timed region
    decode = None
    if not args.no_decode:
        sel = json.load(open(os.path.join(REPO, "data", "selected_heads.json")))["nq__llama3"]["heads"]
        prompts, ws = [], []
        for j in range(args.decode_batch):
            rec = nq[(rank * args.decode_batch + j) % len(nq)]
            _, enc, w, _ = spans.encode(tok, name, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                        [0.1, 1, 1, 1, 1], "")
            prompts.append(enc["input_ids"][0].to(dev))
            ws.append(w)
        eng.generate(prompts[:2], ws[:2], sel, max_new_tokens=4)          # warm the graph path
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        td = time.perf_counter()
        eng.generate(prompts, ws, sel, max_new_tokens=args.decode_tokens, eos_ids=(), use_graph=True,
                     stop_on_eos=False)
        torch.cuda.synchronize()
        dt = torch.tensor([time.perf_counter() - td], device=dev, dtype=torch.float64)
        if world > 1:
            torch.distributed.all_reduce(dt, op=torch.distributed.ReduceOp.MAX)
        decode = {"metric": "questions/sec reweighted-decode", "value": world * args.decode_batch / float(dt.item()),
                  "unit": "questions/s", "batch_per_gpu": args.decode_batch, "new_tokens": args.decode_tokens,
                  "heads": "nq/llama3 selected_heads top-894", "scores": "ideal [0.1,1,1,1,1]",
                  "seconds": float(dt.item()), "note": "prefill + graph-replayed greedy steps, EOS ignored (random weights)"}
        log(f"[rank {rank}] decode: {decode['value']:.2f} questions/s")

    # ---------------- CPU baseline: the reference hook path on the host cores (rank 0, N = 1 only)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.model == "llama3-8b":
        from oracle import cpu_baseline
        t0 = time.time()
        model = cpu_baseline.hf_model_from_engine(eng)
        qi, ids, w, ans = work[0]
        units_s = [(0, 0), (L - 1, H - 1), (L // 2, 3), (1, 7)][:args.cpu_units]
        r = cpu_baseline.time_ie_units(model, ids.cpu(), w, ans.cpu(), units_s)
        cpu = {"value": r["units_per_s"], "unit": "heads/s", "cores": r["cores"], "kind": "port",
               "sample": f"{r['units']} IE units (hooked full forward + full-vocab logits + .item(), "
                         f"re_weighting.py:162-171) of NQ question {qi} at T'={ids.numel()}, after 1 un-hooked "
                         f"forward; {r['seconds']:.1f}s; bf16 torch CPU; extrapolates linearly per unit"}
        del model
        log(f"[rank 0] cpu baseline {cpu['value']:.4f} heads/s on {cpu['cores']} cores ({time.time() - t0:.0f}s)")

    if rank == 0:
        roof = None
        if kt is not None and kt["total_ms"] > 0:
            ach = kt["flops"] / (kt["total_ms"] * 1e-3) / 1e12
            roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": None,
                    "kernel": "cram_prefill (credibility-biased causal GQA flash attention, bf16 MFMA)",
                    "launches": kt["launches"], "avg_launch_ms": round(kt["avg_ms"], 4),
                    "hbm_gbs_algorithmic": round(kt["bytes"] / (kt["total_ms"] * 1e-3) / 1e9, 1),
                    "flops_per_launch": kt["flops"] / kt["launches"]}
        step_tf = flops_all / elapsed / 1e12
        out = {
            "metric": METRIC, "value": round(heads_per_s, 3), "unit": "heads/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic: random-init Llama-3-8B weights; rebuilt NQ-1000 prompts via offline BPE tokenizer",
            "config": {"workload": "Llama-3-8B Find_Best_Heads IE sweep, 32 layers x 32 heads per question, "
                                   "scores [0,1,1,1,1], 1 NQ question per GPU per step",
                       "model": args.model, "questions_per_step": world, "mean_prompt_tokens": round(mean_T, 1),
                       "parallelism": f"dp{world} question-sharded + RCCL all-gather of IE"},
            "roofline": roof,
            "step_roofline": {"bound": "mfma", "achieved": round(step_tf, 2), "peak": PEAK_BF16_TFLOPS * world,
                              "unit": "TFLOP/s", "frac": round(step_tf / (PEAK_BF16_TFLOPS * world), 4),
                              "flops_per_question": flops_all / max(1, world * args.steps)},
            "cpu_baseline": cpu,
            "decode": decode,
        }
        if cpu:
            out["speedup_vs_cpu"] = round(heads_per_s / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
