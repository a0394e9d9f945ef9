"""Multi-process (gloo, world_size 2) tests of the IE-sweep sharding and the final all-gather.

The GPU path runs the same code with backend "nccl" (RCCL over xGMI); here the
kernels are the CPU stand-ins of tests/cpu_ops.py.
"""
import gzip
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from cram_amd import dist as cdist


def test_lpt_and_snake():
    costs = [9, 1, 5, 5, 3, 7, 2]
    bins = cdist.lpt_shards(costs, 3)
    assert sorted(i for b in bins for i in b) == list(range(7))
    loads = [sum(costs[i] for i in b) for b in bins]
    assert max(loads) - min(loads) <= 2
    sn = cdist.snake_layers(32, 8)
    assert sorted(l for b in sn for l in b) == list(range(32))
    cost = [sum(32 - l for l in b) for b in sn]        # work of layer l ~ L - l
    assert max(cost) - min(cost) <= 8
    assert cdist.lpt_shards([1.0], 4)[1:] == [[], [], []]


def test_gather_rows_single_process():
    local = torch.arange(6.0).view(2, 3)
    out = cdist.gather_rows(local, torch.tensor([3, 0]), 4)
    assert torch.equal(out[3], local[0]) and torch.equal(out[0], local[1]) and out[1].abs().sum() == 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, root, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from transformers import AutoModelForCausalLM, AutoTokenizer
    from cram_amd import spans, sweep
    from cram_amd.engine import CrAMEngine
    from tests import cpu_ops
    from tests import tiny_models as tm
    r, w, _ = cdist.init("gloo")
    assert (r, w) == (rank, world)
    path = os.path.join(root, "Qwen2-tiny")
    tok = AutoTokenizer.from_pretrained(path)
    eng = CrAMEngine.from_hf(AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval())
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        nq = json.load(f)[:3]
    inputs = []
    for rec in nq:
        _, enc, wt, _ = spans.encode(tok, path, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                     [0, 1, 1, 1, 1], rec["wrong_answer"])
        ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
        inputs.append((enc["input_ids"][0], wt[0], ans))
    with cpu_ops.patched_ops():
        full = cdist.sweep_questions(lambda i: sweep.ie_question(eng, *inputs[i]), len(inputs),
                                     [x[0].numel() for x in inputs], (eng.spec.num_layers, eng.spec.num_heads),
                                     torch.device("cpu"))
    if rank == 0:
        np.save(out_path, full.numpy())
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_two_rank_sweep_matches_single_process(tmp_path):
    from tests import tiny_models as tm
    root = str(tmp_path)
    tm.save_model("qwen2", root)
    out = str(tmp_path / "ie2.npy")
    mp.spawn(_worker, args=(2, _free_port(), root, out), nprocs=2, join=True)
    two = np.load(out)
    # single-process reference of the same three questions
    from transformers import AutoModelForCausalLM, AutoTokenizer
    from cram_amd import spans, sweep
    from cram_amd.engine import CrAMEngine
    from tests import cpu_ops
    path = os.path.join(root, "Qwen2-tiny")
    tok = AutoTokenizer.from_pretrained(path)
    eng = CrAMEngine.from_hf(AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval())
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        nq = json.load(f)[:3]
    one = []
    with cpu_ops.patched_ops():
        for rec in nq:
            _, enc, wt, _ = spans.encode(tok, path, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                         [0, 1, 1, 1, 1], rec["wrong_answer"])
            ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
            one.append(sweep.ie_question(eng, enc["input_ids"][0], wt[0], ans).numpy())
    np.testing.assert_array_equal(two, np.stack(one))
    assert np.abs(two).sum() > 0
