#!/usr/bin/env python3
"""Diagnostic: a world-1 HIP-IPC transport (every round still exports its buffers' IPC handles), one plan, a few
rounds, then the plan destroyed and re-created on the same transport and a few more rounds.  Prints each step's
outcome (the failing buffer's pointer / allocation / size when an export fails)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import torch  # noqa: E402

from omr import Layout, cdist, ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    L = Layout(n=2 << 20, block_size=256)
    eng = cdist.CppSparseAllreduce(L, dev, transport="ipc", uid=cdist.ipc_unique_id(), rank=0, world=1)
    x = ops.fill_blocks(torch.from_numpy(ops.gen_bitmap(0, 0.2, L.nb)).to(dev), L)
    for step in range(3):
        for r in range(3):
            try:
                eng.run(x, out=x.clone(), mode=int(os.environ.get("MODE", "0")))
                torch.cuda.synchronize()
                print(f"plan {step} round {r}: ok", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"plan {step} round {r}: {e}", flush=True)
                return 1
        eng.replan()
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
