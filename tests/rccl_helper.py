"""Subprocess body of tests/test_gpu_rccl.py: the RCCL ("nccl" backend) process group and the
collectives bench.py runs at N > 1 (verdict-word all-gather, max-over-ranks all-reduce,
barrier), on one GPU with world size 1."""
import os
import sys

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", sys.argv[1])
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
w = torch.arange(1 << 14, dtype=torch.int64, device="cuda")
allw = torch.empty_like(w)
dist.all_gather_into_tensor(allw, w)
t = torch.tensor([3.5], dtype=torch.float64, device="cuda")
dist.all_reduce(t, op=dist.ReduceOp.MAX)
dist.barrier()
torch.cuda.synchronize()
ok = bool((allw == w).all()) and float(t.item()) == 3.5
dist.destroy_process_group()
print("RCCL_OK" if ok else "RCCL_MISMATCH")
