#!/usr/bin/env python3
"""Host cost of HIP launches / events (tools/launch_cost.hip, lc_run) in the contexts the round runs in: a bare
process with torch and the GPU initialised; after torch.distributed's RCCL group (world 1, eager init); after a
CppSparseAllreduce engine (two more RCCL communicators, the round's streams and events) has run rounds; and while
a second host thread polls hipEventQuery as RCCL's proxy thread does.
usage: torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/launch_cost_ctx.py [gloo|nccl]
(gloo: torch.distributed's group is gloo, so the only RCCL communicators are the engine's)"""
import ctypes
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import torch  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "build", "liblaunch_cost.so"))


def run(tag):
    print(f"## {tag}", flush=True)
    lib.lc_run()


torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
run("torch + GPU initialised")
pg = sys.argv[1] if len(sys.argv) > 1 else "nccl"
if pg == "nccl":
    torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", 0))
else:
    torch.distributed.init_process_group("gloo")
run(f"+ torch.distributed {pg} group (world 1)")
from omr import Layout, cdist, ops  # noqa: E402
L = Layout.from_bytes(256 << 20, 256)
x = ops.fill_blocks(torch.from_numpy(ops.gen_bitmap(0, 0.095, L.nb)).cuda(), L)
out = x.clone()
eng = cdist.CppSparseAllreduce(L, device=torch.device("cuda", 0))
for _ in range(20):
    eng.run(x, out=out, mode=1, async_=True, defer=True)
eng.join(torch.cuda.current_stream())
torch.cuda.synchronize()
run("+ round engine (2 RCCL communicators, plan / comm streams) after 20 rounds")
eng.run(x, out=out, mode=1, async_=True, defer=True, thread=True)
eng.join(torch.cuda.current_stream())
torch.cuda.synchronize()
run("+ the engine's progress thread started (idle)")
eng.close()
torch.distributed.destroy_process_group()
