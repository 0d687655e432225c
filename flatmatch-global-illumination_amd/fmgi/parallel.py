"""Photon-batch data parallelism across GPUs (one process per GPU, torch.distributed).

The reference has a single OpenCL device (global_illumination_cl.c:279-281). Its launch schedule
flattens into independent work items (gid + rng_offset fully determines a work item's photons,
photonmap.cl:272), so ranks take contiguous, equal shards of the flattened item list -- no data-path
communication -- and the only exchange is one sum-reduce of the per-rank int64 fixed-point lightmaps
(RCCL over xGMI on MI355X nodes, gloo on CPU). Integer addition is associative, so the reduced
lightmap is bit-identical for any world size and any shard split.
"""
from __future__ import annotations


def shard_range(total_items: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [begin, end) of the flattened work-item list for `rank` of `world`
    (sizes differ by at most one item)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    return total_items * rank // world, total_items * (rank + 1) // world


def _host_backend(group) -> bool:
    import torch.distributed as dist

    return dist.get_backend(group) == "gloo"


def reduce_lightmap(lm, dst: int = 0, group=None):
    """Sum the int64 [numTexels, 4] lightmaps of all ranks into rank `dst` (in place there). Device
    tensors go through RCCL; with gloo (CPU tests, rehearsals) they are staged through host memory."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if lm.is_cuda and _host_backend(group):
            host = lm.cpu()
            dist.reduce(host, dst=dst, op=dist.ReduceOp.SUM, group=group)
            if dist.get_rank(group) == dst:
                lm.copy_(host)
        else:
            dist.reduce(lm, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return lm


def gather_rows(row, device=None, group=None):
    """Every rank's row of floats (equal lengths), gathered to every rank in rank order: the per-rank
    timing breakdown bench.py reports at N > 1. float64 so item offsets and photon counts stay exact."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(x) for x in row], dtype=torch.float64, device=device)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return [t.tolist()]
    if t.is_cuda and _host_backend(group):
        t = t.cpu()
    out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return [x.tolist() for x in out]


def all_reduce(t, op, group=None):
    """dist.all_reduce, staging device tensors through host memory on gloo."""
    import torch.distributed as dist

    if t.is_cuda and _host_backend(group):
        host = t.cpu()
        dist.all_reduce(host, op=op, group=group)
        t.copy_(host)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t
