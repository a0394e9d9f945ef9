"""Multi-GPU sharding of the IE sweep: one process per GPU, static work lists, one RCCL all-gather.

The sweep units are independent given the prompt.  The work item is
(question, set of layers): with at least as many questions as ranks, whole
questions are dealt by a static LPT (longest-processing-time-first) assignment on
their token counts (one baseline forward per question); with fewer questions than
ranks — e.g. one question's cal_logits on 8 GPUs — every question's layers are
dealt to all ranks in a snake order (layer l costs ~ L - l suffix layer-forwards),
each rank running the question's baseline forward for its own layers.  No
data-path collective is needed; at the end one `all_gather_into_tensor` (backend
"nccl" = RCCL over xGMI on MI355X, "gloo" in the CPU tests) assembles the fp32 IE
grid [Nq, L, H] on every rank.

Checkpoint / resume (find_best_heads.py:30-40,53-58 resumes by skipping questions
already on file, by index into a fixed input file): with `shard_dir`, every rank
appends one JSON line per finished (question, layer) to its own file
`rank{r}.jsonl` (append-only, fsync'd per work item), keyed by the question's
identity (a hash of question, passages, scores and wrong answer) and a run
fingerprint (model, shapes, logit convention); a restarted run — any world size,
any order or subset of questions — reads every shard file, skips the units whose
(identity, layer) is already there and fills them from disk.  Decode is replica-only (question-sharded,
no collective).
"""
from __future__ import annotations

import glob
import hashlib
import heapq
import json
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init(backend: Optional[str] = None) -> Tuple[int, int, int]:
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def lpt_shards(costs: Sequence[float], world: int) -> List[List[int]]:
    """Static longest-processing-time-first assignment of items (by cost) onto `world` bins."""
    heap = [(0.0, r) for r in range(world)]
    bins: List[List[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        load, r = heapq.heappop(heap)
        bins[r].append(i)
        heapq.heappush(heap, (load + costs[i], r))
    return [sorted(b) for b in bins]


def snake_layers(num_layers: int, world: int) -> List[List[int]]:
    """Layers of ONE question over ranks; cost of layer l ~ (L - l), so deal in a snake order."""
    bins: List[List[int]] = [[] for _ in range(world)]
    for i, l in enumerate(range(num_layers)):
        rnd, pos = divmod(i, world)
        bins[pos if rnd % 2 == 0 else world - 1 - pos].append(l)
    return bins


def _comm_device(t: torch.Tensor, group=None) -> torch.device:
    """Where a collective on `t` must run: gloo only moves host tensors (rehearsal runs on one GPU)."""
    if dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return t.device


def all_reduce_host(t: torch.Tensor, op: str = "sum", group=None) -> torch.Tensor:
    """All-reduce a small tensor with the process group's backend; returns it on t's device."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return t
    x = t.to(_comm_device(t, group))
    dist.all_reduce(x, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX}[op], group=group)
    return x.to(t.device)


def gather_rows(local: torch.Tensor, local_ids: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather per-rank rows (ragged counts) into a dense [n_total, ...] tensor on every rank.

    local: [k, ...] fp32 rows this rank computed; local_ids: [k] int64 global row ids.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        out = torch.zeros((n_total,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        out[local_ids.to(local.device)] = local
        return out
    home = local.device
    dev = _comm_device(local, group)
    local = local.to(dev)
    kmax_t = torch.tensor([local.shape[0]], device=dev, dtype=torch.int64)
    dist.all_reduce(kmax_t, op=dist.ReduceOp.MAX, group=group)
    kmax = int(kmax_t.item())
    row = 1
    for s in local.shape[1:]:
        row *= int(s)
    buf = torch.zeros((kmax, row + 1), dtype=torch.float64, device=dev)
    buf[:, 0] = -1
    buf[:local.shape[0], 0] = local_ids.to(dev, torch.float64)
    buf[:local.shape[0], 1:] = local.reshape(local.shape[0], row).double()   # a rank may hold no rows
    allb = torch.empty((world * kmax, row + 1), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(allb, buf, group=group)
    keep = allb[:, 0] >= 0
    ids = allb[keep, 0].long()
    out = torch.zeros((n_total, row), dtype=torch.float64, device=dev)
    out[ids] = allb[keep, 1:]
    return out.reshape((n_total,) + tuple(local.shape[1:])).to(device=home, dtype=local.dtype)


WorkItem = Tuple[int, List[int]]          # (question index, layers)


def plan(costs: Sequence[float], num_layers: int, world: int) -> List[List[WorkItem]]:
    """Static per-rank work lists [(question, layers)] for the IE sweep (see the module docstring)."""
    nq = len(costs)
    if nq >= world:
        return [[(i, list(range(num_layers))) for i in b] for b in lpt_shards(costs, world)]
    snake = snake_layers(num_layers, world)
    return [[(i, list(snake[r])) for i in range(nq)] if snake[r] else [] for r in range(world)]


def unit_key(*parts) -> str:
    """Identity of one question's units for checkpoint files: a hash of everything that determines its IE rows
    (question, passages, scores, wrong answer).  Resume matches on it, never on the position in the list."""
    return hashlib.sha256(json.dumps(parts, ensure_ascii=False, sort_keys=True).encode("utf-8")).hexdigest()[:24]


def read_shards(shard_dir: str, num_heads: int, run: str = "") -> Dict[Tuple[str, int], List[float]]:
    """{(question key, layer): IE row} from every rank's append-only file, restricted to records of this run
    fingerprint (model, layer / head counts, logit convention); a torn line (a killed writer) is ignored, a later
    line for the same unit wins."""
    done: Dict[Tuple[str, int], List[float]] = {}
    for fn in sorted(glob.glob(os.path.join(shard_dir, "rank*.jsonl"))):
        with open(fn, encoding="utf-8") as f:
            for line in f:
                try:
                    rec = json.loads(line)
                except ValueError:
                    continue
                if (isinstance(rec, dict) and isinstance(rec.get("key"), str) and rec.get("run", "") == run
                        and len(rec.get("ie", ())) == num_heads):
                    done[(rec["key"], int(rec["layer"]))] = [float(x) for x in rec["ie"]]
    return done


class ShardWriter:
    """Append-only per-rank checkpoint file: one line {"key", "run", "layer", "ie", "q"} per finished (question,
    layer); "q" (the position in this run's list) is informational only."""

    def __init__(self, shard_dir: str, rank: int, keys: Sequence[str], run: str = ""):
        os.makedirs(shard_dir, exist_ok=True)
        self.path = os.path.join(shard_dir, f"rank{rank}.jsonl")
        self.keys = list(keys)
        self.run = run
        # a writer killed mid-line left a fragment without its newline: end it, so the next record starts its own
        # line (the fragment stays an unparsable line that read_shards skips)
        if os.path.exists(self.path) and os.path.getsize(self.path) > 0:
            with open(self.path, "rb+") as f:
                f.seek(-1, os.SEEK_END)
                if f.read(1) != b"\n":
                    f.write(b"\n")
                    f.flush()
                    os.fsync(f.fileno())

    def write(self, q: int, layers: Sequence[int], ie_rows) -> None:
        rows = ie_rows.tolist() if hasattr(ie_rows, "tolist") else ie_rows
        lines = []
        for l, row in zip(layers, rows):
            rec = {"key": self.keys[q], "run": self.run, "layer": int(l), "ie": [float(x) for x in row], "q": int(q)}
            lines.append(json.dumps(rec) + "\n")
        with open(self.path, "a", encoding="utf-8") as f:
            f.write("".join(lines))
            f.flush()
            os.fsync(f.fileno())


def sweep_sharded(fn: Callable[[int, List[int]], torch.Tensor], n_questions: int, costs: Sequence[float],
                  num_layers: int, num_heads: int, device, shard_dir: Optional[str] = None, group=None,
                  keys: Optional[Sequence[str]] = None, run: str = "",
                  log: Optional[Callable[[str], None]] = None) -> torch.Tensor:
    """IE [Nq, L, H] (fp32, on `device`, identical on every rank) of n_questions questions.

    fn(i, layers) -> IE rows [len(layers), H] of question i (cram_amd.sweep.ie_question(..., layers=layers)).
    Work is planned by `plan`; with shard_dir, finished units are checkpointed per work item under the question's
    identity keys[i] (unit_key) and the run fingerprint `run`, and a restarted run — any world size, any order or
    subset of questions — reuses exactly the units whose (key, layer) is on disk for the same run.  The rows
    computed in this run travel in ONE all-gather."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if shard_dir and (keys is None or len(keys) != n_questions):
        raise ValueError("checkpointing needs one identity key per question (cram_amd.dist.unit_key)")
    done = read_shards(shard_dir, num_heads, run) if shard_dir else {}
    if shard_dir and world > 1:
        dist.barrier(group)                   # every rank has read the same files before anyone appends
    writer = ShardWriter(shard_dir, rank, keys, run) if shard_dir else None
    rows, ids = [], []
    for q, layers in plan(costs, num_layers, world)[rank]:
        todo = [l for l in layers if not shard_dir or (keys[q], l) not in done]
        if not todo:
            continue
        ie = fn(q, todo).to(device, torch.float32)
        if writer is not None:
            writer.write(q, todo, ie)
        rows.append(ie)
        ids.extend(q * num_layers + l for l in todo)
        if log is not None:
            log(f"[rank {rank}] question {q}: {len(todo)} layers")
    local = torch.cat(rows) if rows else torch.zeros((0, num_heads), dtype=torch.float32, device=device)
    out = gather_rows(local, torch.tensor(ids, dtype=torch.int64), n_questions * num_layers, group)
    if shard_dir:
        for q in range(n_questions):
            for l in range(num_layers):
                row = done.get((keys[q], l))
                if row is not None:
                    out[q * num_layers + l] = torch.tensor(row, dtype=torch.float32, device=out.device)
    return out.view(n_questions, num_layers, num_heads)
