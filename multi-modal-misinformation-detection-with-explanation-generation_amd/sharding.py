"""Data-parallel replicas: one process per GPU, each holding a full weight and
vault replica; a global batch of pairs is cut into contiguous row shards and each rank runs
analyze_batch on its shard.  The forward path has NO collective — rows are independent and the
HIP path is batch-invariant (a row's outputs do not depend on which rows share its batch), so
sharded results are bit-identical to a single-GPU run.  The only communication is the optional
result gather (``gather_rows``), which uses whatever process group the caller set up (RCCL over
xGMI on the node, gloo in tests).
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple

import torch


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, end) rows of `n` for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_rows(local: Dict[str, torch.Tensor], n_total: int, group=None) -> Dict[str, torch.Tensor]:
    """All-gather per-rank row shards (dict of [rows, ...] tensors) back into global row order.
    Shards may be ragged; they are padded to the largest shard for the collective."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    cap = max(e - s for s, e in sizes)
    out = {}
    for k, t in local.items():
        pad = torch.zeros((cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=group)
        out[k] = torch.cat([b[: e - s] for b, (s, e) in zip(bufs, sizes)], dim=0)
    return out


def run_sharded(fn: Callable[[slice], Dict[str, torch.Tensor]], n_total: int, rank: int, world: int,
                gather: bool = True, group=None) -> Dict[str, torch.Tensor]:
    """Apply `fn` (e.g. a closure over Engine.analyze_batch) to this rank's rows; optionally gather."""
    s, e = shard_range(n_total, rank, world)
    local = fn(slice(s, e))
    return gather_rows(local, n_total, group) if gather and world > 1 else local
