"""RCCL rehearsal of the sweep's collective on a one-GPU box: N ranks over backend "nccl" (RCCL), every rank on
cuda:0, each holding a ragged set of fp32 IE rows; cram_amd.dist.gather_rows (the all_reduce + all_gather_into_tensor
the sweep ends with) must return the dense grid bit-exactly on every rank.  Launch:
  python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
      tools/rccl_same_gpu.py
(RCCL may refuse two ranks on one device; the script then reports the error and exits 3.)"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cram_amd import dist as cdist  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    n_total, L, H = 37, 32, 32
    g = torch.Generator().manual_seed(5)
    full = torch.randn(n_total, L, H, generator=g)
    mine = [i for i in range(n_total) if i % world == rank and (i % 7 != 3)]   # ragged: some rows nobody holds
    loc = full[mine].cuda()
    out = cdist.gather_rows(loc, torch.tensor(mine, dtype=torch.int64), n_total)
    torch.cuda.synchronize()
    expect = torch.zeros_like(full)
    held = [i for i in range(n_total) if i % 7 != 3]
    expect[held] = full[held]
    ok = torch.equal(out.cpu(), expect)
    print(f"rank {rank}/{world}: backend {dist.get_backend()} gather_rows {'bit-exact' if ok else 'MISMATCH'} "
          f"({len(mine)} local rows of {n_total})", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)
except Exception as e:  # noqa: BLE001
    print(f"rank {rank}: RCCL with {world} ranks on one device failed: {type(e).__name__}: {e}", flush=True)
    sys.exit(3)
