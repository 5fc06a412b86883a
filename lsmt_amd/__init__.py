"""lsmt_amd — MI355X-native Bloom-filter path for the `cass` LSM store
(mweiden/lsmt, /root/reference/src/bloom.rs).

The HIP extension (lsmt_amd/libcassbloom.so, C ABI in include/cassbloom.h) is
loaded at import; there is no CPU fallback.
"""
from . import _lib

_lib.load()  # fail loudly if the gfx950 extension is not built

from .bloom import (  # noqa: E402
    BloomFilter,
    BloomProto,
    DeviceKeys,
    FilterSet,
    KeyBatch,
    device_count,
    insert_many,
    last_path,
    probe,
    set_dense,
    set_path,
    unpack_hits,
    Table,
    TableMeta,
    get_many,
    sstable_create,
    zone_bounds,
    ZoneMap,
    hits_compress,
    hits_expand,
    hits_expand_set,
)

__all__ = ["BloomFilter", "BloomProto", "DeviceKeys", "FilterSet", "insert_many", "KeyBatch", "device_count", "last_path",
           "probe", "set_dense", "set_path", "unpack_hits", "zone_bounds", "ZoneMap", "TableMeta", "Table", "get_many", "sstable_create",
           "hits_compress", "hits_expand", "hits_expand_set"]
__version__ = "0.1.0"
