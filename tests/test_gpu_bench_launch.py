"""`bench.py --gpus 2` on the real engine: the parent starts two rank processes itself (the
driver's form of the multi-GPU command, mmf_amd.benchrun.launch_ranks), each rank builds its own
engine and host pipeline, times its steps, and the max over ranks gives the whole-job rate.

On a box with one MI355X the two ranks share the card (MMF_BENCH_SHARE_GPU=1: LOCAL_RANK modulo
the device count, gloo for the barrier and the max-over-ranks all-reduce).  The line is tagged as a
rehearsal: this checks the launch, the per-rank engines and the whole-job arithmetic on hardware;
it does not measure scaling."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_on_the_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, MMF_BENCH_SHARE_GPU="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-configs", "--no-per-sample", "--no-e2e", "--no-cpu-baseline", "--no-profile"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["warmup"] == 1
    assert d["config"]["parallelism"].startswith("replicas x2")
    assert "rehearsal" in d["config"]
    # whole-job rate = 2 ranks x 256 pairs x 3 steps / the max-over-ranks time
    assert d["value"] == pytest.approx(2 * 256 * 3 / (d["ms_per_step"] * 3 / 1e3), rel=0.02)


def test_bench_eight_ranks_rehearsal():
    """the driver's 8-GPU command shape, rehearsed on the one-GPU box before the
    first real SCALE run -- `bench.py --gpus 8` starts eight rank processes, each packs and
    calibrates its own engine and host pipeline beside the seven others on the box's host cores,
    and the whole-job line comes back with every rank's engine-build time."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, MMF_BENCH_SHARE_GPU="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3", "--warmup", "1",
           "--no-configs", "--no-per-sample", "--no-e2e", "--no-cpu-baseline", "--no-profile"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["steps"] == 3 and "rehearsal" in d["config"]
    build = d["config"]["engine_build_s_per_rank"]
    print(f"8-rank rehearsal: {d['value']:.0f} pairs/s whole-job (8 ranks on one GPU), engine build per rank {build}")
    assert len(build) == 8 and all(0.0 < b < 300.0 for b in build)
    assert d["value"] == pytest.approx(8 * 256 * 3 / (d["ms_per_step"] * 3 / 1e3), rel=0.02)
