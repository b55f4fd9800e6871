"""One rank of the message-level round over the HIP-IPC transport (omr_msgd_*), launched by tests/test_gpu_msgd.py:
a worker (rank < workers) or a dedicated aggregator.  Saves the worker's result and its wire logs (its messages and
the replies it received, every protocol round of every slot) or the aggregator's replies."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "omnireduce-rdma-demo_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402  (the generator's inputs only)
from omr import Layout, cdist, ops  # noqa: E402


def view(ptr, n, typestr, dev):
    return torch.as_tensor(ops._DeviceView(ptr, (n,), typestr), device=dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--workers", type=int, required=True)
    ap.add_argument("--uid", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--block", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.2)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    L = Layout(n=a.n, block_size=a.block)
    D = cdist.load()
    uid = (ctypes.c_ubyte * cdist.UNIQUE_ID_BYTES).from_buffer_copy(bytes.fromhex(a.uid).ljust(128, b"\0"))
    d, plan = ctypes.c_void_p(), ctypes.c_void_p()
    cdist._check(D.omr_dist_create_ipc(uid, a.rank, a.world, ctypes.byref(d)), "omr_dist_create_ipc")
    cdist._check(D.omr_msgd_plan_create(d, a.workers, L.n, L.block_size, L.num_lanes, L.num_threads,
                                        ctypes.byref(plan)), "omr_msgd_plan_create")
    worker = a.rank < a.workers
    x = out = None
    if worker:  # the reference generator's input: srand(myId+1), 0.01f blocks (client.cc:396-421)
        x = torch.from_numpy(oracle.fill(oracle.gen_bitmap(a.rank, a.density, L.nb), a.block)).to(dev)
    st = torch.cuda.current_stream()
    maxr = ctypes.c_uint32()
    for _ in range(a.rounds):  # every round from the same input (out-of-place)
        if worker:
            out = x.clone()
        cdist._check(D.omr_msgd_round_f32(plan, x.data_ptr() if worker else None, out.data_ptr() if worker else None,
                                          ctypes.byref(maxr), st.cuda_stream), "omr_msgd_round_f32")
    torch.cuda.synchronize()
    G = L.num_threads * 16
    mp, ip, rp, rip, rr = (ctypes.c_void_p() for _ in range(5))
    cap = ctypes.c_uint32()
    who = a.rank if worker else 0
    cdist._check(D.omr_msgd_logs(plan, who, ctypes.byref(mp), ctypes.byref(ip), ctypes.byref(rp), ctypes.byref(rip),
                                 ctypes.byref(rr), ctypes.byref(cap)), "omr_msgd_logs")
    c = cap.value
    res = {"rounds": view(rr.value, G, "<u4", dev).cpu().numpy(), "cap": np.array([c]),
           "maxr": np.array([maxr.value]),
           "reply": view(rp.value, G * c * 2048, "<f4", dev).cpu().numpy().reshape(G, c, 2048),
           "rimm": view(rip.value, G * c, "<u4", dev).cpu().numpy().reshape(G, c)}
    if worker:
        res["out"] = out.cpu().numpy()
        res["msg"] = view(mp.value, G * c * 2048, "<f4", dev).cpu().numpy().reshape(G, c, 2048)
        res["imm"] = view(ip.value, G * c, "<u4", dev).cpu().numpy().reshape(G, c)
    np.savez(a.out, **res)
    D.omr_msgd_plan_destroy(plan)
    D.omr_dist_destroy(d)


if __name__ == "__main__":
    main()
