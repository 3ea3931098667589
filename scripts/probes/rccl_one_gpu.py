"""Probe: the RCCL calls of exchange.py / bench.py on a one-rank "nccl" process group (one GPU):
all_gather_into_tensor of float64 device rows (async), a grouped batch_isend_irecv to the rank
itself into a row slice, all_reduce SUM of float64 and int64 device tensors, barrier.  The
multi-GPU semantics need more ranks; this checks the call signatures, dtypes and views on RCCL."""
import os
import sys

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29555")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
dev = torch.device("cuda", 0)
n = 4096
x = torch.arange(6 * n, dtype=torch.float64, device=dev).reshape(6, n)
# all-gather mode: padded send block -> full table (exchange.py HaloExchange.start / finish)
send = x[:3].clone()
full = torch.zeros((3, n), dtype=torch.float64, device=dev)
w = dist.all_gather_into_tensor(full, send, async_op=True)
w.wait()
ok_ag = torch.equal(full, x[:3])
# p2p mode: grouped isend / irecv of rows straight into a contiguous row slice
buf = torch.index_select(x, 0, torch.tensor([0, 2], device=dev))
dst = x[4:6]
reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, buf, 0), dist.P2POp(dist.irecv, dst, 0)])
for r in reqs:
    r.wait()
ok_p2p = torch.equal(x[4], x[0]) and torch.equal(x[5], x[2])
# statistics all-reduce (float64) and the halo digest table (int64)
s = torch.arange(10, dtype=torch.float64, device=dev)
dist.all_reduce(s, op=dist.ReduceOp.SUM)
t = torch.arange(10, dtype=torch.int64, device=dev) * 7
dist.all_reduce(t, op=dist.ReduceOp.SUM)
m = torch.tensor([3.5], dtype=torch.float64, device=dev)
dist.all_reduce(m, op=dist.ReduceOp.MAX)
dist.barrier()
torch.cuda.synchronize()
ok_ar = torch.equal(s, torch.arange(10, dtype=torch.float64, device=dev)) and \
    torch.equal(t, torch.arange(10, dtype=torch.int64, device=dev) * 7) and float(m.item()) == 3.5
print({"all_gather_into_tensor": ok_ag, "batch_isend_irecv_self": ok_p2p, "all_reduce": ok_ar,
       "backend": dist.get_backend()})
dist.destroy_process_group()
sys.exit(0 if (ok_ag and ok_p2p and ok_ar) else 1)
