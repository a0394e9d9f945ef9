"""The multi-GPU code paths rehearsed on the one-GPU box: several processes share cuda:0, talk
over gloo (two RCCL ranks on one device are refused at communicator setup), and run the product's sharded
sweep and sharded decode on the HIP kernels -- the same cram_amd.dist code the driver's 8-GPU run executes with
backend "nccl".  Every sharded result must equal one process bit for bit:

  * dist.sweep_sharded, world 2 (whole questions by LPT) and world 4 (fewer questions than ranks: each question's
    layers snake-split): the IE grid [Nq, L, H] equals the one-process grid;
  * dist.decode_sharded, world 2: every question decoded exactly once, the gathered answers equal one process
    decoding the same batches.
Reference: RAG_test.py:64-176 (every question once), find_best_heads.py:13-58 (the per-question IE loop).
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

pytestmark = pytest.mark.gpu

KIND = "llama3"
NQ = 3
NDEC = 6
DEC_HEADS = {0: [1, 2], 2: [0], 3: [3]}
DEC_BATCH = 2
NEW = 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(path):
    from transformers import AutoTokenizer
    from cram_amd import spans
    from tests import tiny_models as tm
    tok = AutoTokenizer.from_pretrained(path)
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        nq = json.load(f)[:max(NQ, NDEC)]
    ie, dec = [], []
    for i, rec in enumerate(nq):
        _, enc, wt, _ = spans.encode(tok, path, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                     [0, 1, 1, 1, 1], rec["wrong_answer"])
        ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
        if i < NQ:
            ie.append((enc["input_ids"][0], wt[0], ans))
        _, enc, wt, _ = spans.encode(tok, path, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                     [0.1, 1, 1, 1, 1], "")
        dec.append((enc["input_ids"][0], wt))
    return ie, dec


def _engine(path):
    from transformers import AutoModelForCausalLM
    from cram_amd.engine import CrAMEngine
    model = AutoModelForCausalLM.from_pretrained(path, dtype="auto").to("cuda:0").eval()
    return CrAMEngine.from_hf(model)


def _run_ie(eng, inputs, i, layers):
    from cram_amd import sweep
    ids, w, ans = inputs[i]
    return sweep.ie_question(eng, ids.cuda(), w, ans.cuda(), layers=layers)


def _run_dec(eng, dec, idx):
    return eng.generate([dec[i][0].cuda() for i in idx], [dec[i][1] for i in idx], DEC_HEADS, max_new_tokens=NEW,
                        use_graph=True, stop_on_eos=False)


def _worker(rank, world, port, path, out_path, what):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    torch.distributed.init_process_group("gloo", init_method=f"file://{out_path}.{port}.store", rank=rank,
                                         world_size=world)
    r, w, local = cdist.init("gloo")
    assert (r, w) == (rank, world)
    torch.cuda.set_device(local % torch.cuda.device_count())          # every rank on the one GPU
    eng = _engine(path)
    ie_in, dec = _inputs(path)
    calls = []
    if what == "sweep":
        def fn(i, layers):
            calls.append((i, list(layers)))
            return _run_ie(eng, ie_in, i, layers)
        full = cdist.sweep_sharded(fn, NQ, [x[0].numel() for x in ie_in], eng.spec.num_layers, eng.spec.num_heads,
                                   torch.device("cuda:0"))
        if rank == 0:
            np.save(out_path, full.cpu().numpy())
    else:
        def fn(idx):
            calls.append(list(idx))
            return _run_dec(eng, dec, idx)
        ans = cdist.decode_sharded(fn, NDEC, [float(x[0].numel()) for x in dec], DEC_BATCH)
        with open(f"{out_path}.ans{rank}.json", "w") as f:
            json.dump(ans, f)
    torch.cuda.synchronize()
    with open(f"{out_path}.calls{rank}.json", "w") as f:
        json.dump(calls, f)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.fixture(scope="module")
def tiny(tmp_path_factory, gpu_device):
    from tests import tiny_models as tm
    root = str(tmp_path_factory.mktemp("distgpu"))
    path = tm.save_model(KIND, root)
    eng = _engine(path)
    ie_in, dec = _inputs(path)
    one = np.stack([_run_ie(eng, ie_in, i, None).cpu().numpy() for i in range(NQ)])
    assert np.isfinite(one).all() and np.abs(one).sum() > 0
    del eng
    torch.cuda.empty_cache()
    return path, one, dec


def _spawn(world, path, out, what):
    mp.spawn(_worker, args=(world, _free_port(), path, out, what), nprocs=world, join=True)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_sweep_on_the_gpu_equals_one_process(tmp_path, tiny, world):
    path, one, _ = tiny
    out = str(tmp_path / f"ie{world}.npy")
    _spawn(world, path, out, "sweep")
    np.testing.assert_array_equal(np.load(out), one)
    calls = [json.load(open(f"{out}.calls{r}.json")) for r in range(world)]
    units = sorted((q, l) for c in calls for q, ls in c for l in ls)
    assert units == [(q, l) for q in range(NQ) for l in range(one.shape[1])]        # every unit exactly once
    assert all(calls), "a rank got no work"


def test_sharded_decode_on_the_gpu_answers_each_question_once(tmp_path, tiny):
    path, _, dec = tiny
    world = 2
    out = str(tmp_path / "dec")
    _spawn(world, path, out, "decode")
    calls = [json.load(open(f"{out}.calls{r}.json")) for r in range(world)]
    assert sorted(i for c in calls for b in c for i in b) == list(range(NDEC))
    assert all(len(b) <= DEC_BATCH for c in calls for b in c) and all(calls)
    # one process decoding the same batches (a row's arithmetic depends on its batch's shape, not on the process)
    eng = _engine(path)
    ref = [None] * NDEC
    for c in calls:
        for b in c:
            for i, a in zip(b, _run_dec(eng, dec, b)):
                ref[i] = a
    for r in range(world):
        assert json.load(open(f"{out}.ans{r}.json")) == ref
