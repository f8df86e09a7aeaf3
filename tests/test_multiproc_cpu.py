"""World-size-2 gloo rehearsal of the replica sharding on CPU: every row is
processed by exactly one rank and the gathered result equals the single-process result, bit for
bit.  The per-row compute here is the CPU oracle's FusionJudge (the HIP path needs a GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from mmf_amd.sharding import shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 256, 1001):
        for w in (1, 2, 3, 8):
            rows = []
            for r in range(w):
                s, e = shard_range(n, r, w)
                rows.extend(range(s, e))
            assert rows == list(range(n))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, x, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mmf_amd.weights as W
    from mmf_amd.sharding import run_sharded
    from oracle import models as M, pipeline as P
    sd = M.to_torch(W.generate(W.detector_spec(), 0, [k for k in W.detector_spec() if k.startswith("fusion")]))
    xt = torch.as_tensor(x)

    def fn(sl):
        probs = torch.softmax(P.fusion_logits(sd, xt[sl]), 1)
        return {"probs": probs, "rows": torch.arange(sl.start, sl.stop)}

    res = run_sharded(fn, xt.shape[0], rank, world)
    if rank == 0:
        torch.save({k: v for k, v in res.items()}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [1024, 1001])
def test_gloo_world2_matches_single_process(tmp_path, n):
    import mmf_amd.synthetic as syn
    import mmf_amd.weights as W
    from oracle import models as M, pipeline as P
    x = syn.fusion_inputs(n, 3)
    out = str(tmp_path / "res.pt")
    mp.start_processes(_worker, args=(2, _free_port(), x, out), nprocs=2, join=True, start_method="spawn")
    res = torch.load(out)
    assert res["rows"].tolist() == list(range(n))
    sd = M.to_torch(W.generate(W.detector_spec(), 0, [k for k in W.detector_spec() if k.startswith("fusion")]))
    ref = torch.softmax(P.fusion_logits(sd, torch.as_tensor(x)), 1)
    # row-independent math: the sharded result equals the single-process one bit for bit
    assert torch.equal(res["probs"], ref) or np.allclose(res["probs"].numpy(), ref.numpy(), atol=1e-7)


def _bench_worker(rank, world, port, out_path):
    """bench.py's rank plumbing (mmf_amd.benchrun) over gloo: the launcher's env, per-rank seeds,
    barrier-bracketed timing and the max-over-ranks reduction."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from mmf_amd import benchrun
    w, r, lr = benchrun.rank_env()
    dist = benchrun.init_dist(w, "gloo")
    calls = []
    delay = 0.02 * (r + 1)  # rank 1 is the slow one: the whole-job time must be its time

    def step():
        calls.append(1)
        time.sleep(delay)

    dt = benchrun.timed_steps(step, steps=5, warmup=2, dist=dist)
    rate = benchrun.whole_job_rate(w, 256, 5, dt)
    import torch.distributed as tdist
    rows = [None] * w
    tdist.all_gather_object(rows, {"rank": r, "world": w, "local": lr, "seed": benchrun.input_seed(r),
                                   "calls": len(calls), "dt": dt, "rate": rate})
    if r == 0:
        torch.save(rows, out_path)
    tdist.barrier()
    tdist.destroy_process_group()


def test_benchrun_gloo_world2(tmp_path):
    out = str(tmp_path / "bench.pt")
    mp.start_processes(_bench_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    rows = torch.load(out)
    assert [x["rank"] for x in rows] == [0, 1] and all(x["world"] == 2 for x in rows)
    assert [x["local"] for x in rows] == [0, 1]
    assert len({x["seed"] for x in rows}) == 2  # each rank draws its own shard
    assert all(x["calls"] == 7 for x in rows)  # warmup 2 + exactly 5 timed steps
    # every rank reports the same (max) time, bounded below by the slow rank's 5 x 40 ms
    assert rows[0]["dt"] == rows[1]["dt"] and rows[0]["dt"] >= 5 * 0.04
    assert rows[0]["rate"] == pytest.approx(2 * 256 * 5 / rows[0]["dt"])


def test_benchrun_single_process():
    from mmf_amd import benchrun
    assert benchrun.init_dist(1, "gloo") is None
    assert benchrun.max_over_ranks(1.5) == 1.5
    n = []
    dt = benchrun.timed_steps(lambda: n.append(1), steps=3, warmup=1)
    assert len(n) == 4 and dt >= 0
    assert benchrun.usable_cpus() >= 1


def _run_bench(args, env=None, timeout=180):
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MMF_BENCH_PARENT")}
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py")] + args, env=e, cwd=repo,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p


def test_bench_gpus2_launches_two_ranks():
    """The driver's exact form, `python bench.py --gpus 2` (no launcher): bench.py starts the two
    ranks itself and rank 0's line reports the whole job."""
    rc, res, p = _run_bench(["--gpus", "2", "--steps", "4", "--warmup", "1", "--cpu-standin"])
    assert rc == 0, p.stderr[-2000:]
    assert res["n_gpus"] == 2 and res["config"]["parallelism"].startswith("replicas x2")
    assert res["config"]["rank_launch"] == "bench.py"
    assert res["config"]["global_batch"] == 512 and res["scaling"] == "weak"
    # value = all ranks' pairs / the max-over-ranks time
    assert res["value"] == pytest.approx(2 * 256 * 4 / (res["ms_per_step"] * 4 / 1000), rel=2e-3)
    assert sum(ln.startswith("{") for ln in p.stdout.splitlines()) == 1  # one JSON line


def test_bench_gpus1_is_a_single_process():
    rc, res, p = _run_bench(["--gpus", "1", "--steps", "2", "--warmup", "1", "--cpu-standin"])
    assert rc == 0, p.stderr[-2000:]
    assert res["n_gpus"] == 1 and res["config"]["parallelism"].startswith("replicas x1")
    assert res["config"]["rank_launch"] == "external"  # no child processes were started


def test_bench_failing_rank_fails_the_launch():
    rc, res, p = _run_bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--cpu-standin"],
                            env={"MMF_STANDIN_FAIL_RANK": "1"})
    assert rc != 0 and res is None
    assert "rank 1 exited" in p.stderr
