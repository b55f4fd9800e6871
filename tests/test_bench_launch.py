"""bench.py's launch contract: an N-GPU line is produced only by N ranks on N GPUs.

* `--gpus N > 1` without a launcher starts torch.distributed.run with N ranks as a CHILD process (before any GPU
  call) and relays rank 0's line, or exits non-zero when the node has fewer than N GPUs;
* under a launcher, `--gpus` must equal WORLD_SIZE, and RCCL ranks may not outnumber the GPUs;
* the line's `n_gpus` is the number of GPUs whose ranks ran, `ranks` the number of ranks, and `value` counts the
  bytes all ranks processed (never N x one GPU's rate)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def plan(argv, env, devices):
    return bench.launch_plan(bench.parse(argv), env, devices)


def test_single_gpu_default():
    assert plan([], {}, 1) == ("run", 1)
    assert plan(["--gpus", "1"], {}, 8) == ("run", 1)


def test_gpus_without_launcher_spawns_or_refuses():
    how, what = plan(["--gpus", "8"], {}, 8)
    assert how == "spawn" and what[what.index("--nproc-per-node") + 1] == "8"
    assert "127.0.0.1" in what
    how, msg = plan(["--gpus", "2"], {}, 1)
    assert how == "error" and "1 GPU" in msg
    assert plan(["--gpus", "0"], {}, 8)[0] == "error"
    assert plan(["--gpus", "2", "--workers", "8"], {}, 8)[0] == "error"


@pytest.mark.parametrize("ws", [1, 2, 4, 8])
def test_launched_ranks_are_the_gpus(ws):
    env = {"WORLD_SIZE": str(ws), "RANK": "0", "LOCAL_RANK": "0"}
    assert plan(["--gpus", str(ws)], env, 8) == ("run", ws)
    assert plan([], env, 8) == ("run", ws)  # the launcher's WORLD_SIZE is the rank count
    if ws > 1:
        assert plan(["--gpus", str(ws * 2)], env, 16)[0] == "error"  # --gpus disagrees with the launcher
        assert plan([], env, ws - 1)[0] == "error"                   # two RCCL ranks would share a GPU


def test_ipc_rehearsal_counts_gpus_not_ranks():
    env = {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"}
    assert plan(["--dist-transport", "ipc"], env, 1) == ("run", 1)


def test_cli_refuses_more_gpus_than_present():
    """On this CPU container (0 GPUs) `bench.py --gpus 2` must refuse before measuring anything."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert not any(ln.startswith("{") for ln in p.stdout.splitlines()), p.stdout
    assert "GPU" in p.stderr


@pytest.mark.gpu
def test_gpu_box_refuses_more_gpus_than_present(gpu):
    """On a node with fewer GPUs than asked for, no N-GPU line is printed and the exit code is non-zero."""
    import torch
    n = torch.cuda.device_count() + 1
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0, p.stdout
    assert not any(ln.startswith("{") for ln in p.stdout.splitlines()), p.stdout
    assert f"--gpus {n}" in p.stderr
