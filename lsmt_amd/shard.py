"""Filters shard one subset per GPU; hit bitmaps are exchanged with one
all-gather.

Every rank holds a contiguous subset of the SSTable filters (Database::get's
tables, /root/reference/src/lib.rs:129-134) and probes the full, replicated
key batch against it, producing hit rows [F_local][ceil(n/64)]. Because the
layout is filter-major, rank r's rows are one contiguous slice of the global
[F][ceil(n/64)] bitmap, so the exchange is a plain concatenation. The
exchange itself is the C ABI's (lsmt_amd/csrc/comm.cpp: cb_hits_allgather,
cb_set_probe_allgather_fixed): dense rows, or at BASELINE densities the
set-bit positions of each rank's rows (fixed-size packs) expanded back into
the identical map, with a dense redo on every rank when some rank's pack
overflows. ``Comm`` binds it over one of three transports: RCCL (one process
per GPU, the product path), loopback (every rank in one process, one thread
per rank: tests at world > 1 on one GPU) and a caller-supplied host
all-gather (``Comm.host``: e.g. gloo between processes sharing one GPU).
"""
from __future__ import annotations


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of the filters owned by `rank` (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


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


def comm_shard(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """The C ABI's split (cb_comm_shard): must equal shard_range."""
    import ctypes

    from . import _lib
    lo, cnt = ctypes.c_uint64(), ctypes.c_uint64()
    _lib.check(_lib.load().cb_comm_shard(n_total, world, rank, ctypes.byref(lo), ctypes.byref(cnt)))
    return int(lo.value), int(lo.value + cnt.value)


class Comm:
    """A communicator of the C ABI (cb_comm, lsmt_amd/csrc/comm.cpp): the
    exchange a Rust ``Database::get`` would call over ``extern "C"``
    (INTEGRATION.md), driven here from Python. One process per GPU, ONE
    communicator per rank (pipelined lanes on several streams share it; the
    library runs its collectives in issue order).

    ``Comm.from_process_group(device)`` makes the 128-byte RCCL id on rank 0
    and hands it to the other ranks over the torch.distributed group (any
    channel works: it is only bytes). ``Comm.loopback(world, device)`` gives
    `world` ranks in this process (drive each from its own thread);
    ``Comm.host(rank, world, device, allgather)`` moves the bytes with a
    Python all-gather of host buffers."""

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
        self._keep = None

    @classmethod
    def _adopt(cls, handle: int, keep=None) -> "Comm":
        import ctypes

        from . import _lib
        c = cls.__new__(cls)
        c._L = _lib.load()
        c._h = ctypes.c_void_p(handle)
        r, w, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(c._L.cb_comm_info(c._h, ctypes.byref(r), ctypes.byref(w), ctypes.byref(d)))
        c.rank, c.world, c.device = r.value, w.value, d.value
        c._keep = keep
        return c

    @classmethod
    def loopback(cls, world: int, device: int = 0) -> "list[Comm]":
        """`world` ranks in this process on `device` (cb_comm_init_loopback).
        Rank r's collectives must run on a thread of its own, concurrently
        with the other ranks' (each call returns when every rank made it)."""
        import ctypes

        from . import _lib
        arr = (ctypes.c_void_p * world)()
        _lib.check(_lib.load().cb_comm_init_loopback(world, device, arr))
        return [cls._adopt(arr[r]) for r in range(world)]

    @classmethod
    def host(cls, rank: int, world: int, device: int, allgather) -> "Comm":
        """A communicator whose bytes move through `allgather(send: bytes-like
        numpy uint8 array, recv: numpy uint8 array of world * len(send))`, a
        host-side all-gather the caller provides (cb_comm_init_host)."""
        import ctypes

        import numpy as np

        from . import _lib

        def cb(user, send, recv, nbytes):
            try:
                n = int(nbytes)
                s = np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(send))[:n] if n else \
                    np.zeros(0, np.uint8)
                r = np.ctypeslib.as_array((ctypes.c_uint8 * max(n * world, 1)).from_address(recv))[:n * world] \
                    if n else np.zeros(0, np.uint8)
                allgather(s, r)
                return 0
            except Exception:  # reported to the library as a failed transport
                import traceback
                traceback.print_exc()
                return 1

        fn = _lib.HOST_ALLGATHER_FN(cb)
        h = ctypes.c_void_p()
        _lib.check(_lib.load().cb_comm_init_host(rank, world, device, fn, None, ctypes.byref(h)))
        return cls._adopt(h.value, keep=fn)

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

    def abort(self) -> int:
        """cb_comm_abort: end the communicator from any thread (a watchdog),
        also while another thread is blocked in one of its collectives.
        Returns the C status (0 on success)."""
        if getattr(self, "_h", None) is None or not self._h.value:
            return 0
        return int(self._L.cb_comm_abort(self._h))

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
        fixed-size packs -> expand; with ok=None an overflow is detected on
        the host and the batch redone densely, with ok (an int32 device tensor
        holding 1) it is reported there instead. Returns whether the map came
        from the packs."""
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
