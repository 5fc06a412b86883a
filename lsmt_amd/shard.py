"""Filters shard one subset per GPU; hit bitmaps are exchanged with one
all-gather.

Every rank holds a contiguous subset of the SSTable filters (Database::get's
tables, /root/reference/src/lib.rs:129-134) and probes the full, replicated
key batch against it, producing hit rows [F_local][ceil(n/64)]. Because the
layout is filter-major, rank r's rows are one contiguous slice of the global
[F][ceil(n/64)] bitmap, so the exchange is a plain concatenation:
``all_gather_into_tensor`` over RCCL/xGMI on GPUs (gloo on CPU in the tests).
Uneven shards are padded to the largest shard and sliced back.
"""
from __future__ import annotations


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of the filters owned by `rank` (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_hits(local_hits, n_total: int, group=None, out=None):
    """All-gather every rank's hit rows into the global [n_total][words] bitmap
    (rows in global filter order). local_hits: [F_local][words] int64 tensor."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rows = max(shard_range(n_total, world, r)[1] - shard_range(n_total, world, r)[0] for r in range(world))
    words = local_hits.shape[1]
    even = all(shard_range(n_total, world, r)[1] - shard_range(n_total, world, r)[0] == rows
               for r in range(world))
    if even:
        full = out if out is not None else torch.empty((n_total, words), dtype=local_hits.dtype,
                                                       device=local_hits.device)
        dist.all_gather_into_tensor(full, local_hits.contiguous(), group=group)
        return full
    pad = torch.zeros((rows, words), dtype=local_hits.dtype, device=local_hits.device)
    pad[: local_hits.shape[0]] = local_hits
    buf = torch.empty((world * rows, words), dtype=local_hits.dtype, device=local_hits.device)
    dist.all_gather_into_tensor(buf, pad, group=group)
    parts = []
    for r in range(world):
        lo, hi = shard_range(n_total, world, r)
        parts.append(buf[r * rows: r * rows + (hi - lo)])
    full = torch.cat(parts, 0)
    if out is not None:
        out.copy_(full)
        return out
    return full
