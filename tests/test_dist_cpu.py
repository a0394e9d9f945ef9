"""Multi-process (gloo) tests of the IE-sweep sharding, checkpoint / resume and the final all-gather.

The GPU path runs the same code with backend "nccl" (RCCL over xGMI); here the kernels are the CPU stand-ins of
tests/cpu_ops.py.  Every sharded result must equal the single-process sweep bit for bit:
  * world 2, 3 questions: whole questions dealt by LPT;
  * world 4 and 8, 3 questions (fewer questions than ranks): every question's layers snake-split over the ranks
    (cal_logits of one question on several GPUs);
  * resume after a kill: a world-4 run whose rank 1 dies after its first work item (the spawner then tears the
    others down mid-flight), restarted at world 2 from the per-rank shard files — the restart computes only the
    units missing on disk (find_best_heads.py:30-40,53-58 resume semantics, at (question, layer) granularity).
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

KIND = "llama3"          # tiny Llama-3: 4 layers x 4 heads (GQA 2:1)
NQ = 3


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


def test_plan_covers_every_unit_once():
    for nq, L, world in [(1, 32, 8), (3, 32, 8), (8, 32, 8), (1000, 32, 8), (5, 4, 2), (3, 4, 8), (1, 28, 3)]:
        p = cdist.plan([100 + (i * 37) % 11 for i in range(nq)], L, world)
        assert len(p) == world
        units = [(q, l) for items in p for q, ls in items for l in ls]
        assert sorted(units) == [(q, l) for q in range(nq) for l in range(L)]
    # one question on 8 ranks: every rank gets layers, snake-balanced (cost of layer l ~ L - l)
    p = cdist.plan([900.0], 32, 8)
    loads = [sum(32 - l for _, ls in items for l in ls) for items in p]
    assert min(loads) > 0 and max(loads) - min(loads) <= 8


def test_gather_rows_single_process():
    local = torch.arange(6.0).view(2, 3)
    out = cdist.gather_rows(local, torch.tensor([3, 0]), 4)
    assert torch.equal(out[3], local[0]) and torch.equal(out[0], local[1]) and out[1].abs().sum() == 0


KEYS = ["qa", "qb", "qc"]


def test_shard_files_tolerate_a_torn_line(tmp_path):
    w = cdist.ShardWriter(str(tmp_path), 0, KEYS)
    w.write(2, [0, 3], torch.tensor([[1.5, -2.0], [0.25, 3.0]]))
    with open(tmp_path / "rank0.jsonl", "a") as f:
        f.write('{"key": "qc", "run": "", "layer": 1, "ie": [0.1')       # a writer killed mid-line
    cdist.ShardWriter(str(tmp_path), 1, KEYS).write(1, [1], [[7.0, 8.0]])
    done = cdist.read_shards(str(tmp_path), 2)
    assert done == {("qc", 0): [1.5, -2.0], ("qc", 3): [0.25, 3.0], ("qb", 1): [7.0, 8.0]}
    # the SAME rank restarts after the torn line: its next record must not be glued onto the fragment
    cdist.ShardWriter(str(tmp_path), 0, KEYS).write(0, [2], [[4.0, 5.0]])
    done = cdist.read_shards(str(tmp_path), 2)
    assert done[("qa", 2)] == [4.0, 5.0] and len(done) == 4


def test_resume_matches_question_identity_not_position(tmp_path):
    """A restart over a reordered / different question list reuses only the units of the same questions, and only
    from the same run fingerprint (find_best_heads.py:30-40 resumes by index into a fixed file; here lists vary)."""
    d = str(tmp_path)
    calls = []

    def fn(i, layers, tag):
        calls.append((tag, i, tuple(layers)))
        return torch.tensor([[float(ord(tag[0])) * 100 + i * 10 + l, -1.0] for l in layers])

    first = ["qa", "qb", "qc"]
    out1 = cdist.sweep_sharded(lambda i, ls: fn(i, ls, first[i]), 3, [1.0, 1.0, 1.0], 2, 2, torch.device("cpu"),
                               shard_dir=d, keys=first, run="m1")
    assert len(calls) == 3
    calls.clear()
    second = ["qc", "qx", "qa"]                  # reordered, one new question
    out2 = cdist.sweep_sharded(lambda i, ls: fn(i, ls, second[i]), 3, [1.0, 1.0, 1.0], 2, 2, torch.device("cpu"),
                               shard_dir=d, keys=second, run="m1")
    assert calls == [("qx", 1, (0, 1))]          # only the new question is computed
    assert torch.equal(out2[0], out1[2]) and torch.equal(out2[2], out1[0])
    calls.clear()
    cdist.sweep_sharded(lambda i, ls: fn(i, ls, second[i]), 3, [1.0, 1.0, 1.0], 2, 2, torch.device("cpu"),
                        shard_dir=d, keys=second, run="m2")
    assert len(calls) == 3                       # another run fingerprint reuses nothing
    with pytest.raises(ValueError):
        cdist.sweep_sharded(lambda i, ls: fn(i, ls, "q"), 1, [1.0], 2, 2, torch.device("cpu"), shard_dir=d)


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
        nq = json.load(f)[:NQ]
    out = []
    for rec in nq:
        _, enc, wt, _ = spans.encode(tok, path, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                     [0, 1, 1, 1, 1], rec["wrong_answer"])
        ans = tok([rec["wrong_answer"]], return_tensors="pt")["input_ids"][0, 1:]
        out.append((enc["input_ids"][0], wt[0], ans))
    return out


def _keys(inputs):
    return [cdist.unit_key(ids.tolist(), w.float().tolist(), a.tolist()) for ids, w, a in inputs]


def _worker(rank, world, port, root, out_path, shard_dir, die_after):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from transformers import AutoModelForCausalLM
    from cram_amd import sweep
    from cram_amd.engine import CrAMEngine
    from tests import cpu_ops
    from tests import tiny_models as tm
    torch.distributed.init_process_group("gloo", init_method=f"file://{out_path}.{port}.store", rank=rank,
                                         world_size=world)             # file rendezvous: no port race under xdist
    r, w, _ = cdist.init("gloo")
    assert (r, w) == (rank, world)
    path = os.path.join(root, tm.DIR_NAME[KIND])
    eng = CrAMEngine.from_hf(AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval())
    inputs = _inputs(path)
    calls = []

    def fn(i, layers):
        if die_after is not None and rank == die_after[0] and len(calls) == die_after[1]:
            os._exit(3)                                      # killed between two work items
        calls.append((i, list(layers)))
        return sweep.ie_question(eng, *inputs[i], layers=layers)

    with cpu_ops.patched_ops():
        full = cdist.sweep_sharded(fn, len(inputs), [x[0].numel() for x in inputs], eng.spec.num_layers,
                                   eng.spec.num_heads, torch.device("cpu"), shard_dir=shard_dir, keys=_keys(inputs))
    with open(f"{out_path}.calls{rank}.json", "w") as f:
        json.dump(calls, f)
    if rank == 0:
        np.save(out_path, full.numpy())
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.fixture(scope="module")
def single(tmp_path_factory):
    """Single-process sweep of the same questions (the bar for every sharded run)."""
    from transformers import AutoModelForCausalLM
    from cram_amd import sweep
    from cram_amd.engine import CrAMEngine
    from tests import cpu_ops
    from tests import tiny_models as tm
    root = str(tmp_path_factory.mktemp("dist"))
    path = tm.save_model(KIND, root)
    eng = CrAMEngine.from_hf(AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval())
    with cpu_ops.patched_ops():
        one = np.stack([sweep.ie_question(eng, *x).numpy() for x in _inputs(path)])
    assert np.abs(one).sum() > 0
    return root, one


def _spawn(root, world, out, shard_dir=None, die_after=None):
    mp.spawn(_worker, args=(world, _free_port(), root, out, shard_dir, die_after), nprocs=world, join=True)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_sweep_matches_single_process(tmp_path, single, world):
    root, one = single
    out = str(tmp_path / f"ie{world}.npy")
    _spawn(root, world, out)
    np.testing.assert_array_equal(np.load(out), one)
    calls = [json.load(open(f"{out}.calls{r}.json")) for r in range(world)]
    units = sorted((q, l) for c in calls for q, ls in c for l in ls)
    assert units == [(q, l) for q in range(NQ) for l in range(one.shape[1])]      # every unit exactly once
    if world > NQ:                                                                 # layer split of each question
        assert all(len(ls) < one.shape[1] for c in calls for _, ls in c)


def test_resume_after_kill(tmp_path, single):
    root, one = single
    shards = str(tmp_path / "shards")
    out = str(tmp_path / "ie.npy")
    with pytest.raises(Exception):
        _spawn(root, 4, out, shard_dir=shards, die_after=(1, 1))
    keys = _keys(_inputs(os.path.join(root, __import__("tests.tiny_models").tiny_models.DIR_NAME[KIND])))
    done = {(keys.index(k), l): row for (k, l), row in cdist.read_shards(shards, one.shape[2]).items()}
    assert 0 < len(done) < NQ * one.shape[1]
    for (q, l), row in done.items():                       # what reached the disk is final
        np.testing.assert_array_equal(np.asarray(row, dtype=np.float32), one[q, l])
    _spawn(root, 2, out, shard_dir=shards)
    np.testing.assert_array_equal(np.load(out), one)
    calls = [json.load(open(f"{out}.calls{r}.json")) for r in range(2)]
    redone = {(q, l) for c in calls for q, ls in c for l in ls}
    assert not redone & set(done), "a unit on disk was recomputed"
    assert len(redone) + len(done) == NQ * one.shape[1]
    assert len(cdist.read_shards(shards, one.shape[2])) == NQ * one.shape[1]


# ---------------------------------------------------------------------------------------------------------------
# question-sharded decode (replicas only; RAG_test.py:64-176 answers every question exactly once)
# ---------------------------------------------------------------------------------------------------------------
NDEC = 6
DEC_HEADS = {0: [1, 2], 2: [0], 3: [3]}
DEC_LENS = (200, 137, 171, 150, 188, 120)


def test_decode_batches_balance():
    costs = [float(c) for c in (5, 1, 9, 3, 7, 2, 8)]
    b = cdist.decode_batches(range(7), costs, 3)
    assert [len(x) for x in b] == [3, 2, 2]                      # ceil(7 / 3) = 3 near-equal batches
    assert [i for x in b for i in x] == sorted(range(7), key=lambda i: costs[i])
    assert cdist.decode_batches([], costs, 4) == []
    assert [len(x) for x in cdist.decode_batches(range(1000), [1.0] * 1000, 512)] == [500, 500]


def _dec_inputs(path):
    from transformers import AutoTokenizer
    from cram_amd import spans
    from tests import tiny_models as tm
    tok = AutoTokenizer.from_pretrained(path)
    with gzip.open(os.path.join(tm.REPO, "data", "nq_1000.json.gz"), "rt") as f:
        nq = json.load(f)[:NDEC]
    out = []
    for rec, L in zip(nq, DEC_LENS):
        _, enc, wt, _ = spans.encode(tok, path, rec["question"], rec["ori_fake"] + rec["reranked_dense_ctxs"],
                                     [0.1, 1, 1, 1, 1], "")
        out.append((enc["input_ids"][0, :L], wt[:, :L]))
    return out


def _dec_worker(rank, world, port, root, out_path, shard_dir, die_after):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from transformers import AutoModelForCausalLM
    from cram_amd.engine import CrAMEngine
    from tests import cpu_ops
    from tests import tiny_models as tm
    # rendezvous through a file next to the outputs (no TCP port to race for under pytest-xdist), then cdist.init
    # reads rank / world from the torch.distributed.run environment as under the launcher
    torch.distributed.init_process_group("gloo", init_method=f"file://{out_path}.{port}.store", rank=rank, world_size=world)
    cdist.init("gloo")
    path = os.path.join(root, tm.DIR_NAME[KIND])
    eng = CrAMEngine.from_hf(AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval())
    inputs = _dec_inputs(path)
    calls = []

    def fn(idx):
        if die_after is not None and rank == die_after[0] and len(calls) == die_after[1]:
            os._exit(3)                                          # killed between two decode batches
        calls.append(list(idx))
        return eng.generate([inputs[i][0] for i in idx], [inputs[i][1] for i in idx], DEC_HEADS, max_new_tokens=4,
                            use_graph=False)

    keys = [cdist.unit_key(ids.tolist(), w.float().tolist()) for ids, w in inputs]
    with cpu_ops.patched_ops():
        ans = cdist.decode_sharded(fn, NDEC, [float(x[0].numel()) for x in inputs], 2, shard_dir=shard_dir,
                                   keys=keys, run="tiny-decode")
    with open(f"{out_path}.calls{rank}.json", "w") as f:
        json.dump(calls, f)
    with open(f"{out_path}.ans{rank}.json", "w") as f:
        json.dump(ans, f)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.fixture(scope="module")
def dec_single(single):
    """One process, one batch: the answers every sharded decode must reproduce."""
    from transformers import AutoModelForCausalLM
    from cram_amd.engine import CrAMEngine
    from tests import cpu_ops
    from tests import tiny_models as tm
    root, _ = single
    path = os.path.join(root, tm.DIR_NAME[KIND])
    eng = CrAMEngine.from_hf(AutoModelForCausalLM.from_pretrained(path, dtype="auto").eval())
    inputs = _dec_inputs(path)
    with cpu_ops.patched_ops():
        ref = eng.generate([x[0] for x in inputs], [x[1] for x in inputs], DEC_HEADS, max_new_tokens=4,
                           use_graph=False)
    return root, ref


def _dec_spawn(root, world, out, shard_dir=None, die_after=None):
    mp.spawn(_dec_worker, args=(world, _free_port(), root, out, shard_dir, die_after), nprocs=world, join=True)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_decode_answers_each_question_once(tmp_path, dec_single, world):
    root, ref = dec_single
    out = str(tmp_path / f"dec{world}")
    _dec_spawn(root, world, out)
    calls = [json.load(open(f"{out}.calls{r}.json")) for r in range(world)]
    decoded = sorted(i for c in calls for b in c for i in b)
    assert decoded == list(range(NDEC))                          # every question exactly once across ranks
    assert all(len(b) <= 2 for c in calls for b in c)            # batches of at most `batch` rows
    assert sum(1 for c in calls if c) == min(world, NDEC)        # every rank got work
    for r in range(world):                                        # the full answer list on every rank
        assert json.load(open(f"{out}.ans{r}.json")) == ref


def test_sharded_decode_resume_after_kill(tmp_path, dec_single):
    root, ref = dec_single
    shards = str(tmp_path / "answers")
    out = str(tmp_path / "dec")
    with pytest.raises(Exception):
        _dec_spawn(root, 2, out, shard_dir=shards, die_after=(1, 1))
    done = cdist.read_answers(shards, "tiny-decode")
    assert 0 < len(done) < NDEC
    _dec_spawn(root, 2, out, shard_dir=shards)
    calls = [json.load(open(f"{out}.calls{r}.json")) for r in range(2)]
    redone = [i for c in calls for b in c for i in b]
    assert len(redone) + len(done) == NDEC                       # nothing on file is decoded again
    assert json.load(open(f"{out}.ans0.json")) == ref
