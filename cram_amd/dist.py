"""Multi-GPU sharding of the IE sweep: one process per GPU, static work lists, one RCCL all-gather.

The sweep units are independent given the prompt.  Questions are
dealt to ranks by a static LPT (longest-processing-time-first) assignment on
their token counts, so no data-path collective is needed; at the end one
`all_gather_into_tensor` (backend "nccl" = RCCL over xGMI on MI355X, "gloo" in
the CPU tests) assembles the fp32 IE grid [Nq, L, H] on every rank.  Decode is
replica-only (question-sharded, no collective).
"""
from __future__ import annotations

import heapq
import os
from typing import List, Optional, Sequence, Tuple

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
    row = int(torch.tensor(local.shape[1:]).prod().item()) if local.dim() > 1 else 1
    buf = torch.zeros((kmax, row + 1), dtype=torch.float64, device=dev)
    buf[:, 0] = -1
    buf[:local.shape[0], 0] = local_ids.to(dev, torch.float64)
    buf[:local.shape[0], 1:] = local.reshape(local.shape[0], -1).double()
    allb = torch.empty((world * kmax, row + 1), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(allb, buf, group=group)
    keep = allb[:, 0] >= 0
    ids = allb[keep, 0].long()
    out = torch.zeros((n_total, row), dtype=torch.float64, device=dev)
    out[ids] = allb[keep, 1:]
    return out.reshape((n_total,) + tuple(local.shape[1:])).to(device=home, dtype=local.dtype)


def sweep_questions(fn, n_questions: int, costs: Sequence[float], row_shape: Tuple[int, ...], device,
                    group=None) -> torch.Tensor:
    """Run fn(i) -> IE row_shape for this rank's LPT share of questions and all-gather [Nq, *row_shape]."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    mine = lpt_shards(costs, world)[rank]
    res = [fn(i).to(device, torch.float32) for i in mine]
    local = torch.stack(res) if res else torch.zeros((0,) + tuple(row_shape), dtype=torch.float32, device=device)
    return gather_rows(local, torch.tensor(mine, dtype=torch.int64), n_questions, group)
