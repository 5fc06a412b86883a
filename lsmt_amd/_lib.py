"""Loads the HIP extension ``lsmt_amd/libcassbloom.so`` (C ABI in
``include/cassbloom.h``) with ctypes.

There is no fallback: if the shared library is missing or cannot be loaded,
importing the product API raises. Build it with ``__graft_entry__.build()`` or
``make -C lsmt_amd/csrc``.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libcassbloom.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "cassbloom.h")

CB_OK = 0
CB_EINVAL = -1
CB_EZEROM = -2
CB_ENOMEM = -3
CB_EHIP = -4
CB_EDECODE = -5
CB_ENODEV = -6
CB_EUTF8 = -7

PATH_AUTO, PATH_DIRECT, PATH_TILED = 0, 1, 2
XCHG_DENSE, XCHG_SPARSE = 0, 1
COMM_ID_BYTES = 128
# cb_host_allgather_fn (include/cassbloom.h): int (*)(void* user, const void* send, void* recv, uint64_t bytes)
HOST_ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint64)

_lib = None


class CassBloomError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"cassbloom error {code}: {msg}")
        self.code = code


class ExtensionMissing(ImportError):
    pass


class ZoneBounds(ctypes.Structure):
    """struct cb_zone_bounds (include/cassbloom.h)."""
    _fields_ = [("min", ctypes.c_void_p), ("min_len", ctypes.c_uint64), ("has_min", ctypes.c_int),
                ("max", ctypes.c_void_p), ("max_len", ctypes.c_uint64), ("has_max", ctypes.c_int)]


class MetaInfo(ctypes.Structure):
    """struct cb_meta_info (include/cassbloom.h)."""
    _fields_ = [("has_bloom", ctypes.c_int), ("has_zone", ctypes.c_int), ("zone", ZoneBounds)]


def load():
    """Load and prototype the C ABI. Raises ExtensionMissing if not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ExtensionMissing(
            f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C lsmt_amd/csrc` (gfx950 HIP extension; no CPU fallback exists)")
    # torch wheels bundle their own libamdhip64.so.7 (same soname as
    # /opt/rocm's). Whichever loads first serves the whole process, and torch
    # cannot run on a runtime it did not load itself, so when torch is present
    # it is imported first and this library binds to torch's HIP runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P, u8p, u32, u64, i32 = ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    pp = ctypes.POINTER(ctypes.c_void_p)
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    proto = {
        "cb_init": ([i32], i32),
        "cb_device_count": ([ctypes.POINTER(ctypes.c_int)], i32),
        "cb_last_error": ([], ctypes.c_char_p),
        "cb_version": ([], ctypes.c_char_p),
        "cb_stream_synchronize": ([P], i32),
        "cb_stream_release": ([P], i32),
        "cb_host_alloc": ([u64, ctypes.POINTER(P)], i32),
        "cb_host_free": ([P], i32),
        "cb_hits_compress": ([P, u64, u64, P, u64, P], i32),
        "cb_hits_expand": ([P, u32, u64, pu64, u64, u64, P, P, P], i32),
        "cb_hits_pack_words": ([u64, u64, u64, pu64], i32),
        "cb_comm_unique_id": ([P], i32),
        "cb_comm_init": ([i32, i32, P, i32, pp], i32),
        "cb_comm_init_loopback": ([i32, i32, P], i32),
        "cb_comm_init_host": ([i32, i32, i32, HOST_ALLGATHER_FN, P, pp], i32),
        "cb_comm_destroy": ([P], i32),
        "cb_comm_abort": ([P], i32),
        "cb_comm_info": ([P, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)], i32),
        "cb_comm_shard": ([u64, i32, i32, pu64, pu64], i32),
        "cb_hits_allgather": ([P, P, u64, u64, u64, P, i32, u64, P, ctypes.POINTER(i32), P], i32),
        "cb_set_probe_allgather_fixed": ([P, P, u8p, u32, u64, i32, P, u64, P, i32, u64, P, ctypes.POINTER(i32), P],
                                         i32),
        "cb_set_pack_words": ([u64, u64, pu64], i32),
        "cb_set_probe_pack_fixed": ([P, u8p, u32, u64, i32, P, P, u64, P], i32),
        "cb_hits_expand_set": ([P, u32, u64, pu64, u64, u64, P, P, P], i32),
        "cb_filter_create": ([u64, i32, pp], i32),
        "cb_filter_destroy": ([P], i32),
        "cb_filter_bits": ([P, pu64], i32),
        "cb_filter_device": ([P, ctypes.POINTER(ctypes.c_int)], i32),
        "cb_filter_words": ([P, pp, pu64], i32),
        "cb_filter_clear": ([P, P], i32),
        "cb_filter_insert_fixed": ([P, u8p, u32, u64, P], i32),
        "cb_filter_insert_var": ([P, u8p, P, u64, P], i32),
        "cb_filter_insert_fixed_many": ([P, u32, P, u32, P, P], i32),
        "cb_probe_fixed": ([P, u32, u8p, u32, u64, P, P], i32),
        "cb_probe_var": ([P, u32, u8p, P, u64, P, P], i32),
        "cb_may_contain": ([P, u8p, u64, ctypes.POINTER(ctypes.c_int)], i32),
        "cb_filter_host_mirror": ([P, i32], i32),
        "cb_filter_host_mirror_info": ([P, ctypes.POINTER(i32), ctypes.POINTER(i32)], i32),
        "cb_filter_export_bools": ([P, u8p, P], i32),
        "cb_filter_import_bools": ([P, u8p, u64, P], i32),
        "cb_filter_export_packed": ([P, P, P], i32),
        "cb_filter_import_packed": ([P, P, u64, P], i32),
        "cb_filter_to_bytes": ([P, u8p, u64, pu64], i32),
        "cb_filter_from_bytes": ([u8p, u64, i32, pp], i32),
        "cb_set_path": ([i32], i32),
        "cb_last_path": ([], i32),
        "cb_set_create": ([u64, u32, i32, pp], i32),
        "cb_set_destroy": ([P], i32),
        "cb_set_info": ([P, pu64, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)], i32),
        "cb_set_assign": ([P, u32, P, P], i32),
        "cb_set_assign_all": ([P, P, u32, P], i32),
        "cb_set_clear_slot": ([P, u32, P], i32),
        "cb_set_probe_fixed": ([P, u8p, u32, u64, P, P], i32),
        "cb_set_probe_var": ([P, u8p, P, u64, P, P], i32),
        "cb_set_zone": ([P, u32, u8p, u64, i32, u8p, u64, i32, P], i32),
        "cb_set_zone_get": ([P, u32, u8p, u64, pu64, ctypes.POINTER(i32), u8p, u64, pu64,
                             ctypes.POINTER(i32)], i32),
        "cb_set_zone_from_keys_fixed": ([P, u32, u8p, u32, u64, P], i32),
        "cb_set_zone_from_keys_var": ([P, u32, u8p, P, u64, P], i32),
        "cb_zone_bounds_fixed": ([u8p, u32, u64, i32, pu64, pu64, P], i32),
        "cb_zone_bounds_var": ([u8p, P, u64, i32, pu64, pu64, P], i32),
        "cb_meta_encode": ([P, ctypes.POINTER(ZoneBounds), u8p, u64, pu64], i32),
        "cb_meta_decode": ([u8p, u64, i32, pp, ctypes.POINTER(MetaInfo)], i32),
        "cb_set_load_meta": ([P, u32, u8p, u64, P], i32),
        "cb_table_create": ([u8p, u64, i32, P, pp], i32),
        "cb_table_destroy": ([P], i32),
        "cb_table_info": ([P, pu64, pu64], i32),
        "cb_table_lines": ([P, P, P, P], i32),
        "cb_table_data": ([P, pp, pu64], i32),
        "cb_table_copy": ([P, u64, u64, u8p], i32),
        "cb_sstable_create": ([u8p, P, u8p, P, u64, u64, i32, P, pp, pp, pu64, pu64], i32),
        "cb_sstable_create_bounded": ([u8p, P, u64, u8p, P, u64, u64, u64, i32, P, pp, pp], i32),
        "cb_table_wait": ([P], i32),
        "cb_table_zone": ([P, i32, u8p, u64, pu64], i32),
        "cb_table_rebuild": ([P, u64, P, pp, pu64, pu64], i32),
        "cb_table_well_formed": ([P, ctypes.POINTER(i32)], i32),
        "cb_table_force_exact": ([i32], i32),
        "cb_table_bucket_limit": ([u64], i32),
        "cb_set_dense": ([i32], i32),
        "cb_table_search_fixed": ([P, u8p, u32, u64, P, P], i32),
        "cb_table_search_var": ([P, u8p, P, u64, P, P], i32),
        "cb_get_many_fixed": ([P, u32, P, P, u8p, u32, u64, P, P, P, u64, pu64, P], i32),
        "cb_get_many_var": ([P, u32, P, P, u8p, P, u64, P, P, P, u64, pu64, P], i32),
        "cb_set_get_many_fixed": ([P, P, u32, P, u8p, u32, u64, P, P, P, u64, pu64, P], i32),
        "cb_set_get_many_var": ([P, P, u32, P, u8p, P, u64, P, P, P, u64, pu64, P], i32),
        "cb_set_probe_gated_fixed": ([P, u8p, u32, u64, P, P], i32),
        "cb_set_probe_gated_var": ([P, u8p, P, u64, P, P], i32),
        "cb_profile_enable": ([i32], i32),
        "cb_profile_reset": ([], i32),
        "cb_profile_read": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), pu64], i32),
    }
    for name, (args, res) in proto.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != CB_OK:
        msg = load().cb_last_error()
        raise CassBloomError(rc, msg.decode() if msg else "")


def header_symbols() -> list[str]:
    """Every function the public header declares (for the export test)."""
    with open(HEADER_PATH) as fh:
        text = fh.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(cb_\w+)\s*\(", text, re.M)))
