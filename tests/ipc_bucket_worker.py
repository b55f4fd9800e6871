"""One rank of omr_sparse_buckets_f32 over the HIP-IPC transport, its gradient in its own pinned host memory
(launched by tests/test_gpu_buckets.py).  Saves the host buffer after the call."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "omnireduce-rdma-demo_amd"), os.path.join(ROOT, "oracle"), HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import Layout, cdist  # noqa: E402
from test_gpu_buckets import rank_input  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--uid", required=True)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--bucket-mib", type=int, default=8)
    ap.add_argument("--total-mib", type=int, default=32)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    L = Layout.from_bytes(a.bucket_mib << 20, 256)
    total_n = (a.total_mib << 20) // 4
    x, _ = rank_input(a.rank, total_n, L, 0.49, dev)
    host = x.cpu().pin_memory()
    eng = cdist.CppSparseAllreduce(L, dev, transport="ipc", uid=bytes.fromhex(a.uid), rank=a.rank, world=a.world)
    eng.run_buckets(host, mode=a.mode)
    torch.cuda.synchronize()
    np.save(a.out, host.numpy())
    eng.close()


if __name__ == "__main__":
    main()
