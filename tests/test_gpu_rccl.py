"""The RCCL leg of bench.py's multi-GPU timing, run once on the one-GPU box.

An 8-GPU SCALE run times each rank's K steps between `dist.barrier()` calls and takes the max over
ranks with a device-tensor `all_reduce(MAX)` on the "nccl" (RCCL) backend, initialised with
`device_id` (benchrun.init_dist / timed_steps / max_over_ranks).  On one GPU that branch is only
reached at world > 1, so `MMF_BENCH_FORCE_DIST=1` initialises the process group at world 1: the real
bench command then runs the same RCCL calls, and this test checks that it completes and says so.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_rccl_timing_leg_world1():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, MMF_BENCH_FORCE_DIST="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()),
               RANK="0", LOCAL_RANK="0", WORLD_SIZE="1")
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-profile", "--no-configs", "--no-per-sample", "--no-e2e"]
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=240)
    print(r.stderr[-3000:])
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["config"]["timing_collective"].startswith("rccl"), line["config"]
