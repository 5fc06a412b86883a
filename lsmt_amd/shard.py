"""Filters shard one subset per GPU; hit bitmaps are exchanged with one
all-gather.

Every rank holds a contiguous subset of the SSTable filters (Database::get's
tables, /root/reference/src/lib.rs:129-134) and probes the full, replicated
key batch against it, producing hit rows [F_local][ceil(n/64)]. Because the
layout is filter-major, rank r's rows are one contiguous slice of the global
[F][ceil(n/64)] bitmap, so the exchange is a plain concatenation:
``all_gather_into_tensor`` over RCCL/xGMI on GPUs (gloo on CPU in the tests).
Uneven shards are padded to the largest shard and sliced back.

The rows are sparse at BASELINE densities (one table per present key, false
positives ~(1.55 %)^2 per (key, table)), so ``gather_hits_sparse`` ships each
rank's set-bit positions instead (cb_hits_compress -> all-gather of fixed-size
packs -> cb_hits_expand) and rebuilds the identical map; if any rank has more
set bits than the pack holds, every rank sees that in the gathered counts and
all of them take the dense path for that step.
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


def sparse_cap(n_keys: int, f_total: int, world: int) -> int:
    """Pack capacity for a probe batch, the same on every rank (the packs are
    all-gathered as equal-size tensors): sized for the largest shard, with the
    present keys whose table lives on it (half of the SURVEY.md §8d lookups,
    spread over all tables) plus 25 % slack, one false positive per 1000
    (key, table) pairs (the expected rate is 2.4e-4), and 4096."""
    f_local = -(-f_total // world)
    present = (n_keys // 2) * f_local // max(f_total, 1)
    return int(1.25 * present + n_keys * f_local / 1000) + 4096


PACK_BLOCK_WORDS = 2048  # hit words per pack directory entry (exchange.hpp kCompressWords)


def pack_words(nw: int, cap: int) -> int:
    """uint32 words of a pack for nw words of hit rows and cap positions
    (cb_hits_pack_words): {count, 0, positions[cap], directory of one
    {first slot, number} pair per PACK_BLOCK_WORDS words}."""
    return 2 + cap + 2 * -(-nw // PACK_BLOCK_WORDS)


def gather_hits_sparse(local_hits, n_total: int, cap: int, compress, expand, group=None, out=None,
                       stats=None, ok=None):
    """Same result as gather_hits; cap must be equal on every rank
    (sparse_cap). compress(local_hits, pack, cap) fills an int32 pack of
    pack_words(largest shard's words, cap) {count, 0, positions, directory};
    expand(packs, world, row_off, full, ok, cap) rebuilds the global map
    (lsmt_amd.hits_compress / hits_expand on GPUs).

    Synchronous (ok=None): the gathered counts are read on the host; if some
    rank overflowed (the same decision on every rank) all ranks then run the
    dense all-gather, so the result is always complete. stats (a dict,
    optional) receives "sparse" (whether the packs sufficed) and "max_count".

    Asynchronous (ok = an int32 device tensor holding 1): no host round trip;
    expand clears ok if some rank overflowed, and the caller must check ok
    before using the map and redo that batch with gather_hits if it is 0."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    words = local_hits.shape[1]
    stride = pack_words(-(-n_total // world) * words, cap)  # the largest shard's pack, on every rank
    pack = torch.zeros(stride, dtype=torch.int32, device=local_hits.device)
    compress(local_hits, pack, cap)
    packs = torch.empty(world * stride, dtype=torch.int32, device=local_hits.device)
    dist.all_gather_into_tensor(packs, pack, group=group)
    row_off = [shard_range(n_total, world, r)[0] for r in range(world)]
    if ok is not None:
        full = out if out is not None else torch.empty((n_total, words), dtype=local_hits.dtype,
                                                       device=local_hits.device)
        expand(packs, world, row_off, full, ok, cap)
        return full
    counts = packs.view(world, stride)[:, 0].cpu().numpy().astype("int64") & 0xFFFFFFFF
    if stats is not None:
        stats["sparse"] = bool((counts <= cap).all())
        stats["max_count"] = int(counts.max())
    if (counts > cap).any():
        return gather_hits(local_hits, n_total, group=group, out=out)
    full = out if out is not None else torch.empty((n_total, words), dtype=local_hits.dtype,
                                                   device=local_hits.device)
    expand(packs, world, row_off, full, None, cap)
    return full


def comm_shard(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """The C ABI's split (cb_comm_shard): must equal shard_range."""
    import ctypes

    from . import _lib
    lo, cnt = ctypes.c_uint64(), ctypes.c_uint64()
    _lib.check(_lib.load().cb_comm_shard(n_total, world, rank, ctypes.byref(lo), ctypes.byref(cnt)))
    return int(lo.value), int(lo.value + cnt.value)


class Comm:
    """An RCCL communicator of the C ABI (cb_comm, lsmt_amd/csrc/comm.cpp):
    the exchange a Rust ``Database::get`` would call over ``extern "C"``
    (INTEGRATION.md), driven here from Python. One process per GPU.

    ``Comm.from_process_group(device)`` makes the 128-byte id on rank 0 and
    hands it to the other ranks over the torch.distributed group (any
    channel works: it is only bytes)."""

    def __init__(self, rank: int, world: int, device: int, uid: bytes):
        import ctypes

        from . import _lib
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError("the communicator id is 128 bytes")
        self._L = _lib.load()
        self._h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * len(uid)).from_buffer_copy(uid)
        _lib.check(self._L.cb_comm_init(rank, world, ctypes.addressof(buf), device, ctypes.byref(self._h)))
        self.rank, self.world, self.device = rank, world, device

    @staticmethod
    def unique_id() -> bytes:
        import ctypes

        from . import _lib
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
        _lib.check(_lib.load().cb_comm_unique_id(ctypes.addressof(buf)))
        return bytes(buf)

    @classmethod
    def from_process_group(cls, device: int, group=None) -> "Comm":
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls(rank, world, device, obj[0])

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.cb_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def allgather(self, local_hits, n_total: int, out, sparse: bool = False, cap: int = 0, ok=None,
                  stream=None) -> bool:
        """out ([n_total][words] int64 device tensor) := every rank's hit rows
        (cb_hits_allgather). local_hits: this rank's [rows][words] slice
        (rows = its shard_range of n_total). sparse: compress -> all-gather of
        (2 + cap)-word packs -> expand; with ok=None an overflow is detected
        on the host and the batch redone densely, with ok (an int32 device
        tensor holding 1) it is reported there instead. Returns whether the
        map came from the packs."""
        import ctypes

        from . import _lib
        from .bloom import _ptr_of, _stream
        rows, words = local_hits.shape
        if tuple(out.shape) != (n_total, words):
            raise ValueError("out must be [n_total][words]")
        lp, k1 = _ptr_of(local_hits)
        fp, k2 = _ptr_of(out)
        op, k3 = _ptr_of(ok)
        used = ctypes.c_int(0)
        _lib.check(self._L.cb_hits_allgather(self._h, lp, rows, words, n_total, fp,
                                             _lib.XCHG_SPARSE if sparse else _lib.XCHG_DENSE, cap, op,
                                             ctypes.byref(used), _stream(stream)))
        return bool(used.value)

    def probe_allgather(self, fset, keys, n_total: int, local_out, out, sparse: bool = False, cap: int = 0,
                        ok=None, gated: bool = False, stream=None) -> bool:
        """This rank's FilterSet probe and the exchange in one C call
        (cb_set_probe_allgather_fixed): keys uint8[n, key_len] on the device;
        local_out [used][ceil(n/64)] and out [n_total][ceil(n/64)] int64
        device tensors. In sparse mode the probe kernel writes the pack
        itself. Returns whether the map came from the packs."""
        import ctypes

        from . import _lib
        from .bloom import _ptr_of, _stream
        n = int(keys.shape[0])
        kp, k1 = _ptr_of(keys)
        lp, k2 = _ptr_of(local_out)
        fp, k3 = _ptr_of(out)
        op, k4 = _ptr_of(ok)
        used = ctypes.c_int(0)
        _lib.check(self._L.cb_set_probe_allgather_fixed(
            self._h, fset._h, kp, int(keys.shape[1]), n, int(bool(gated)), lp, n_total, fp,
            _lib.XCHG_SPARSE if sparse else _lib.XCHG_DENSE, cap, op, ctypes.byref(used), _stream(stream)))
        return bool(used.value)
