"""Rank plumbing of the benchmark (bench.py), factored out so that the multi-process path runs in
the CPU test suite exactly as it runs on an 8-GPU node (tests/test_multiproc_cpu.py::
test_benchrun_gloo_world2 drives these functions over a gloo world of 2 with a CPU stand-in engine).

One process per GPU: torchrun / torch.distributed.run sets RANK, LOCAL_RANK, WORLD_SIZE and
MASTER_*, or `bench.py --gpus N` started directly becomes the parent of N rank processes itself
(`launch_ranks`, before anything touches the GPU); the batch is sharded by rank with no collective
on the data path:
every rank times its own steps, the barrier brackets the timed region, and the whole-job time is
the MAX over ranks (one all_reduce of one float) -- the only collective traffic.
"""
from __future__ import annotations

import math
import os
import sys
import time
from typing import Callable, Optional

import torch

INPUT_SEED = 1234  # inputs seeded 1234 + rank


def rank_env() -> tuple:
    """(world, rank, local_rank) from the launcher's environment (1, 0, 0 when run directly)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def needs_launch(n: int) -> bool:
    """`bench.py --gpus N` started directly (no launcher environment) with N > 1: this process
    becomes the parent of N rank processes instead of running a step itself."""
    return n > 1 and "WORLD_SIZE" not in os.environ


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, cmd: list, check_devices: bool = True, poll_s: float = 0.2) -> int:
    """Run `cmd` as N rank processes on this node, the way torch.distributed.run would: each child
    gets RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = N and MASTER_ADDR / MASTER_PORT
    (127.0.0.1, a free port).  The parent never touches the GPU (no HIP call, so no exec or fork
    hazard after device initialisation; `torch.cuda.device_count()` does not initialise HIP on this
    image); it relays rank 0's stdout (the JSON line) and returns the first non-zero child exit
    code, terminating the other ranks, or 0 when every rank succeeded."""
    import subprocess
    import threading
    if check_devices:
        have = torch.cuda.device_count()
        if have < n:
            progress(f"--gpus {n}: only {have} HIP device(s) visible")
            return 2
    env0 = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    procs = []
    import signal

    def stop_children(signum, _frame):  # the launcher itself stopped (e.g. a driver timeout): no orphans
        for p in procs:
            if p.poll() is None:
                p.terminate()
        sys.exit(128 + signum)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, stop_children)
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr))

    def relay():
        for line in procs[0].stdout:
            sys.stdout.write(line.decode())
            sys.stdout.flush()
    t = threading.Thread(target=relay, daemon=True)
    t.start()
    rc = 0
    live = set(range(n))
    stop_at = None
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                progress(f"rank {r} exited with {c}: stopping the other ranks")
                for q in live:
                    procs[q].terminate()
                stop_at = time.monotonic()
        if stop_at is not None and time.monotonic() - stop_at > 30:
            for q in live:  # a rank stuck in a collective ignores SIGTERM
                procs[q].kill()
        time.sleep(poll_s)
    t.join(timeout=10)
    return rc


def input_seed(rank: int) -> int:
    """Each rank draws its own shard of the synthetic workload."""
    return INPUT_SEED + rank


def init_dist(world: int, backend: str, device: Optional[torch.device] = None, force: bool = False):
    """torch.distributed with `backend` ("nccl" = RCCL over xGMI on the GPU node, "gloo" in the CPU
    tests) when world > 1, else None.  force: initialise it at world 1 too (MMF_BENCH_FORCE_DIST=1:
    the one-GPU box runs the RCCL branch -- device_id binding, barrier, device all_reduce(MAX) --
    that an 8-GPU SCALE run takes, tests/test_gpu_rccl.py)."""
    if world <= 1 and not force:
        return None
    for k, v in (("MASTER_ADDR", "127.0.0.1"), ("RANK", "0"), ("WORLD_SIZE", str(world))):
        os.environ.setdefault(k, v)
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(free_port())
    import torch.distributed as dist
    if backend == "nccl":
        dist.init_process_group(backend, device_id=device)
    else:
        dist.init_process_group(backend)
    return dist


def timed_steps(step: Callable[[], None], steps: int, warmup: int, dist=None,
                sync: Callable[[], None] = lambda: None, device: Optional[torch.device] = None) -> float:
    """`warmup` untimed steps, then exactly `steps` timed steps bracketed by a barrier and a device
    synchronisation on both sides; returns the MAX over ranks of the timed wall time (seconds)."""
    for _ in range(warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    return max_over_ranks(dt, dist, device)


def max_over_ranks(x: float, dist=None, device: Optional[torch.device] = None) -> float:
    if not dist:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_per_rank(x: float, world: int, rank: int, dist=None, device: Optional[torch.device] = None) -> list:
    """[x of rank 0, x of rank 1, ...] on every rank (a SUM all-reduce of one-hot slots)."""
    if not dist:
        return [x]
    t = torch.zeros(world, dtype=torch.float64, device=device)
    t[rank] = x
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.cpu()]


def whole_job_rate(world: int, units_per_rank_step: int, steps: int, seconds: float) -> float:
    """Units all ranks processed / whole-job time (weak scaling: per-rank work fixed)."""
    return world * units_per_rank_step * steps / seconds


def usable_cpus() -> int:
    """Host cores this process may actually run on: its affinity set, capped by a cgroup CPU quota
    and by OMP_NUM_THREADS when either is set (a container's share of a large host can show every
    CPU of the machine in the affinity mask; the GPU pool states its per-GPU share that way)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:  # cgroup v2: "<quota> <period>" or "max <period>"
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        try:  # cgroup v1
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                n = min(n, max(1, math.ceil(q / per)))
        except (OSError, ValueError):
            pass
    return n


def progress(msg: str) -> None:
    """One line to stderr per bench phase (the JSON result stays the only stdout line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)
