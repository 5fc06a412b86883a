"""GPU parity for SURVEY.md §8f row 4: SsTable::create on the device — stable
sort, `key \\t base64(value) \\n` formatting, the table's Bloom filter and zone
map — byte-exact against the golden fixtures and the C oracle.

Reference: src/sstable.rs:51-87 (create), src/memtable.rs:34-41 (sorted
scan), src/lib.rs:195-210 (flush).
"""
import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu


def test_create_golden(gpu, golden):
    for name, c in golden["create"].items():
        entries = [(bytes.fromhex(k), bytes.fromhex(v)) for k, v in zip(c["keys_hex"], c["values_hex"])]
        t, bloom, zone = gpu.sstable_create(entries)
        assert t.data().hex() == c["file_hex"], name
        # the table is indexed and searchable, and its filter/zone are the
        # ones SsTable::create builds next to the file
        o = oracle.OracleFilter(1024)
        oz = oracle.OracleZone()
        for k, _ in entries:
            o.insert(k)
            oz.update(k)
        assert np.array_equal(bloom.bools(), o.bools()), name
        assert (zone.min, zone.max) == oz.bounds, name
        ot = oracle.OracleTable(bytes.fromhex(c["file_hex"]))
        assert t.nlines == ot.nlines, name


@pytest.mark.parametrize("n,sorted_input", [(1, True), (1000, True), (1000, False), (200_003, False),
                                            (200_003, True)])
def test_create_random_vs_oracle(gpu, n, sorted_input):
    rng = np.random.default_rng(n)
    keys = workload.key_range(3000 + n, n)
    if sorted_input:
        keys = workload.sort_keys16(keys)  # memtable scan order: the sort is skipped
    vlen = rng.integers(0, 40, n)
    voff = np.zeros(n + 1, np.uint64)
    np.cumsum(vlen, out=voff[1:])
    vdata = rng.integers(0, 256, int(voff[-1]) + 1, dtype=np.uint8)
    koff = np.arange(0, 16 * (n + 1), 16, dtype=np.uint64)
    kb = gpu.KeyBatch(n=n, data=np.ascontiguousarray(keys.reshape(-1)), offsets=koff)
    vb = gpu.KeyBatch(n=n, data=vdata, offsets=voff)
    t, bloom, zone = gpu.sstable_create((kb, vb), m=1 << 20)
    entries = [(bytes(keys[i]), vdata[voff[i]:voff[i + 1]].tobytes()) for i in range(n)]
    assert t.data() == oracle.sstable_create(entries)
    assert t.well_formed and t.nlines == n
    o = oracle.OracleFilter(1 << 20)
    o.insert_fixed(keys)
    assert np.array_equal(bloom.bools(), o.bools())
    srt = workload.sort_keys16(keys)
    assert (zone.min, zone.max) == (bytes(srt[0]), bytes(srt[-1]))
    # round trip through the read path: every key finds its own value
    look = keys[rng.integers(0, n, min(n, 5000))]
    which, voffs, vals = gpu.get_many([t], look)
    assert (which == 0).all()
    pos = {bytes(k): i for i, k in enumerate(keys)}
    for j in range(0, len(look), 97):
        i = pos[bytes(look[j])]
        assert vals[voffs[j]:voffs[j + 1]] == vdata[voff[i]:voff[i + 1]].tobytes()


def _same_index(gpu, t, probes):
    # the index written straight from the entries equals the one built by
    # re-reading the file (cb_table_create), and searches agree with the oracle
    r = gpu.Table(t.data())
    for a, b in zip(t.lines(), r.lines()):
        assert np.array_equal(a, b)
    assert t.nlines == r.nlines and t.well_formed == r.well_formed
    ot = oracle.OracleTable(t.data())
    d = np.frombuffer(b"".join(probes) or b"\0", np.uint8)
    offs = np.zeros(len(probes) + 1, np.uint64)
    np.cumsum([len(k) for k in probes], out=offs[1:])
    kb = gpu.KeyBatch(n=len(probes), data=d, offsets=offs)
    exp = [ot.search(k)[0] for k in probes]
    assert list(t.search(kb)) == exp and list(r.search(kb)) == exp


@pytest.mark.parametrize("sorted_input", [True, False])
def test_create_direct_index(gpu, sorted_input):
    rng = np.random.default_rng(11)
    keys = [bytes(rng.integers(32, 127, rng.integers(0, 30), dtype=np.uint8)).replace(b"\t", b"_")
            for _ in range(5000)]
    keys = sorted(set(keys)) if sorted_input else list(dict.fromkeys(keys))
    vals = [bytes(rng.integers(0, 256, rng.integers(0, 50), dtype=np.uint8)) for _ in keys]
    t, _, _ = gpu.sstable_create(list(zip(keys, vals)))
    assert t.data() == oracle.sstable_create(list(zip(keys, vals)))
    assert t.well_formed and t.nlines == len(keys)
    _same_index(gpu, t, keys[::7] + [b"zz" * 20, b"", b"\x00"])


def test_create_keys_with_line_breaks_and_tabs(gpu):
    # keys holding '\n' / '\t' split lines / keys differently in the file than
    # in the entry list: the table is then indexed from the file, as
    # SsTable::get splits it (src/sstable.rs:142-146)
    keys = [b"a", b"b\tc", b"d\ne", b"f", b"g\n", b"\th", b"i"]
    vals = [bytes([i]) * i for i in range(len(keys))]
    t, _, _ = gpu.sstable_create(list(zip(keys, vals)))
    assert t.data() == oracle.sstable_create(list(zip(keys, vals)))
    assert t.nlines == oracle.OracleTable(t.data()).nlines != len(keys)
    _same_index(gpu, t, keys + [b"b", b"d", b"e", b"g", b"", b"h"])


def test_create_short_keys_stable_sort(gpu):
    # unsorted keys of 0..16 bytes, compared from their sort records alone:
    # duplicates keep their input order, trailing NULs order after the shorter
    # key ("a" < "a\0"), shared 8- and 16-byte prefixes
    rng = np.random.default_rng(13)
    base = [b"", b"a", b"a\x00", b"a\x00\x00", b"abcdefgh", b"abcdefgh\x00", b"abcdefghA", b"\xff" * 16,
            b"\xff" * 15, b"0123456789abcdef", b"0123456789abcdee"]
    base += [bytes(rng.integers(0, 256, rng.integers(0, 17), dtype=np.uint8)) for _ in range(200)]
    keys = [base[i] for i in rng.integers(0, len(base), 30_000)]
    vals = [i.to_bytes(3, "little") for i in range(len(keys))]
    t, bloom, zone = gpu.sstable_create(list(zip(keys, vals)))
    assert t.data() == oracle.sstable_create(list(zip(keys, vals)))
    assert (zone.min, zone.max) == (min(keys), max(keys))


def test_create_ragged_duplicates(gpu):
    # ragged keys with many duplicates and shared prefixes (longer than 16
    # bytes too): the rocPRIM merge sort must be stable and order by full key
    rng = np.random.default_rng(9)
    base = [bytes(rng.integers(97, 99, rng.integers(0, 24), dtype=np.uint8)) for _ in range(300)]
    keys = [base[i] for i in rng.integers(0, len(base), 20_000)]
    vals = [i.to_bytes(4, "little") for i in range(len(keys))]
    t, bloom, zone = gpu.sstable_create(list(zip(keys, vals)))
    assert t.data() == oracle.sstable_create(list(zip(keys, vals)))
    assert not t.well_formed  # duplicate keys: the exact search trajectory is used
    assert (zone.min, zone.max) == (min(keys), max(keys))


@pytest.mark.parametrize("on_device", [False, True])
def test_create_zone_keys_long_and_device(gpu, on_device):
    # zone bounds come back with the table (cb_table_zone): keys longer than
    # the 256 bytes carried inline take one extra copy; inputs on the host or
    # in HBM give the same table, filter and bounds
    import torch
    rng = np.random.default_rng(21)
    keys = [bytes(rng.integers(97, 123, int(rng.integers(1, 600)), dtype=np.uint8)) for _ in range(3000)]
    keys = list(dict.fromkeys(keys))
    keys[5] = b"\x00" + b"a" * 700     # smallest, longer than the inline bytes
    keys[9] = b"\xff" * 300 + b"z"     # largest
    vals = [bytes(rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8)) for _ in keys]
    kd = np.frombuffer(b"".join(keys), np.uint8)
    ko = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=ko[1:])
    vd = np.frombuffer(b"".join(vals) + b"\0", np.uint8)
    vo = np.zeros(len(vals) + 1, np.uint64)
    np.cumsum([len(v) for v in vals], out=vo[1:])
    if on_device:
        kd, vd = torch.from_numpy(kd.copy()).cuda(), torch.from_numpy(vd.copy()).cuda()
        ko, vo = torch.from_numpy(ko.view(np.int64)).cuda(), torch.from_numpy(vo.view(np.int64)).cuda()
    kb = gpu.KeyBatch(n=len(keys), data=kd, offsets=ko)
    vb = gpu.KeyBatch(n=len(vals), data=vd, offsets=vo)
    t, bloom, zone = gpu.sstable_create((kb, vb), m=1 << 16)
    assert t.data() == oracle.sstable_create(list(zip(keys, vals)))
    assert (zone.min, zone.max) == (min(keys), max(keys))
    o = oracle.OracleFilter(1 << 16)
    for k in keys:
        o.insert(k)
    assert np.array_equal(bloom.bools(), o.bools())


def test_table_zone_only_for_created_tables(gpu):
    # cb_table_zone answers for tables SsTable::create made with entries; a
    # table indexed from an existing file, or an empty one, has no bounds
    from lsmt_amd._lib import CassBloomError
    t, _, zone = gpu.sstable_create([(b"b", b"1"), (b"a", b"2")])
    assert (t._zone(0), t._zone(1)) == (b"a", b"b") == (zone.min, zone.max)
    with pytest.raises(CassBloomError):
        gpu.Table(t.data())._zone(0)
    e, _, ez = gpu.sstable_create([])
    assert ez.min is None and ez.max is None
    with pytest.raises(CassBloomError):
        e._zone(1)


@pytest.mark.parametrize("n,shape", [(2, "random"), (2047, "random"), (2048, "descending"), (2049, "random"),
                                     (4095, "random"), (4096, "descending"), (4097, "equal"), (8193, "random"),
                                     (6145, "equal"), (70_001, "long"), (300_001, "random"),
                                     (1 << 20, "descending"), (1_300_000, "random"), (20_000, "hot"),
                                     (100_000, "skew"),
                                     (50_000, "text")])
def test_create_sort_sizes(gpu, n, shape):
    """The hand-written stable sorts of unsorted flush batches (sort.hip):
    the bin sort for n > 4096 (one binning pass over the directory map's
    buckets, one LDS sort per group: 1024-record group sorts up to ~1.18M
    entries, 2048-record ones above) and, below that or when a group outgrows
    an LDS tile, the merge sort (LDS block sorts of 4096 records, then
    merge-path rounds). Random keys, reversed keys, all-equal keys (pure
    stability; one bin: the fallback), long keys sharing 16-byte prefixes
    (the fallback), one key repeated 6000 times among random ones (a hot bin:
    the fallback), 90 % of the keys under one 4-byte prefix (skewed bins) and
    'user'+digits text keys; the file must equal the oracle's stable sort +
    format (src/sstable.rs:57-72)."""
    rng = np.random.default_rng(n)
    if shape == "equal":
        keys = [b"same-key"] * n
    elif shape == "hot":
        keys = [bytes(r) for r in workload.key_range(6000 + n, n)]
        for i in rng.choice(n, 6000, replace=False):
            keys[i] = b"0123456789abcdef"
    elif shape == "skew":
        keys = [bytes(r) for r in workload.key_range(7000 + n, n)]
        for i in rng.choice(n, 9 * n // 10, replace=False):
            keys[i] = b"aaaa" + keys[i][4:]
    elif shape == "text":
        keys = [b"user%012d" % int(x) for x in rng.integers(0, 10 ** 9, n)]
    elif shape == "long":
        pre = [bytes(rng.integers(97, 100, 16, dtype=np.uint8)) for _ in range(7)]
        keys = [pre[i % 7] + bytes(rng.integers(97, 99, rng.integers(0, 12), dtype=np.uint8)) for i in range(n)]
    else:
        k = workload.key_range(5000 + n, n)
        if shape == "descending":
            k = workload.sort_keys16(k)[::-1]
        keys = [bytes(r) for r in k]
        if shape == "random":  # some duplicates and short keys mixed in
            for i in rng.integers(0, n, n // 10):
                keys[i] = keys[rng.integers(0, n)][: rng.integers(0, 17)]
    vals = [(i % 65536).to_bytes(2, "little") for i in range(n)]
    t, _, zone = gpu.sstable_create(list(zip(keys, vals)))
    assert t.data() == oracle.sstable_create(list(zip(keys, vals)))
    assert (zone.min, zone.max) == (min(keys), max(keys))


def test_create_bin_overflow_over_stale_workspace(gpu):
    """A bin sort that overflows (two 8-byte key prefixes, 100K keys each: a
    bin far larger than an LDS tile) right after a larger flush on the same
    stream, whose sort records and value spans (longer values, other offsets)
    still sit in the workspace. The overflowed groups leave their slice of
    those buffers unwritten, so the first k_format must not run over them
    (ADVICE r3): the file must equal the oracle's, and a table made before it
    must be untouched (src/sstable.rs:57-72)."""
    rng = np.random.default_rng(77)
    big = [bytes(r) for r in workload.key_range(9100, 300_000)]
    big_vals = [bytes(rng.integers(0, 256, 60, dtype=np.uint8)) for _ in big]
    t_big, _, _ = gpu.sstable_create(list(zip(big, big_vals)))
    neighbour = [(bytes(r), b"v%d" % i) for i, r in enumerate(workload.key_range(9200, 5000))]
    t_nb, _, _ = gpu.sstable_create(neighbour)
    nb_file = t_nb.data()
    tail = workload.key_range(9300, 200_000)
    keys = [(b"aaaaaaaa" if i % 2 else b"bbbbbbbb") + bytes(r[:8]) for i, r in enumerate(tail)]
    vals = [(i % 251).to_bytes(1, "little") for i in range(len(keys))]
    t, _, zone = gpu.sstable_create(list(zip(keys, vals)))
    assert t.data() == oracle.sstable_create(list(zip(keys, vals)))
    assert (zone.min, zone.max) == (min(keys), max(keys))
    assert t_nb.data() == nb_file == oracle.sstable_create(neighbour)
    assert t_big.nlines == len(big)


@pytest.mark.parametrize("n", [1 << 22, 1 << 24])
def test_create_unsorted_large(gpu, n):
    """Unsorted flushes at 4M entries and at 2^24, the largest batch the bin
    sort takes (10923 groups of 2048-record sorts, 4096 count blocks), with
    BASELINE's 16-B keys and values: the whole file against a numpy
    restatement of the sort + format (workload.sstable_bytes; the keys are
    distinct, so the stable order is the key order), the zone bounds, and a
    sample of keys through the read path (src/sstable.rs:57-72,133-179)."""
    keys = workload.key_range(8000 + n, n)
    vals = workload.table_value(keys, 3)
    koff = np.arange(0, 16 * (n + 1), 16, dtype=np.uint64)
    kb = gpu.KeyBatch(n=n, data=np.ascontiguousarray(keys.reshape(-1)), offsets=koff)
    vb = gpu.KeyBatch(n=n, data=np.ascontiguousarray(vals.reshape(-1)), offsets=koff)
    t, _, zone = gpu.sstable_create((kb, vb), m=1 << 20)
    want = workload.sstable_bytes(keys, vals)
    got = np.frombuffer(t.data(), np.uint8)
    assert got.size == want.size and np.array_equal(got, want)
    w = keys.view(">u8").reshape(n, 2)
    lo, hi = np.lexsort((w[:, 1], w[:, 0]))[[0, -1]]
    assert (zone.min, zone.max) == (bytes(keys[lo]), bytes(keys[hi]))
    rng = np.random.default_rng(n)
    idx = rng.integers(0, n, 4096)
    which, voffs, out = gpu.get_many([t], keys[idx])
    assert (np.asarray(which) == 0).all()
    got_vals = np.frombuffer(bytes(out), np.uint8).reshape(-1, 16)
    assert np.array_equal(got_vals, vals[idx])


def _dev_batches(keys, vals):
    import torch
    kd = torch.from_numpy(np.frombuffer(b"".join(keys) or b"\0", np.uint8).copy()).cuda()
    vd = torch.from_numpy(np.frombuffer(b"".join(vals) or b"\0", np.uint8).copy()).cuda()
    ko = np.zeros(len(keys) + 1, np.int64)
    np.cumsum([len(k) for k in keys], out=ko[1:])
    vo = np.zeros(len(vals) + 1, np.int64)
    np.cumsum([len(v) for v in vals], out=vo[1:])
    return (torch.from_numpy(ko).cuda(), kd), (torch.from_numpy(vo).cuda(), vd)


@pytest.mark.parametrize("shape", ["sorted", "unsorted", "two_prefixes", "one_prefix", "small"])
def test_create_enqueue_only_then_finalise(gpu, shape):
    """cb_sstable_create only enqueues (the device picks: no sort for a sorted
    batch, the bin sort, or — for keys the bins cannot split — a merge sort
    when the table is finalised). Five tables in flight on one stream, none
    waited for until all are queued; every file, zone and filter must equal
    the oracle's (src/sstable.rs:51-87)."""
    import torch
    rng = np.random.default_rng(len(shape))
    st = torch.cuda.Stream()
    made, want = [], []
    for r in range(5):
        n = 300 if shape == "small" else 60_000
        base = [bytes(x) for x in workload.key_range(9500 + 10 * r + len(shape), n)]
        if shape == "two_prefixes":
            keys = [(b"ns:user:" if i % 2 else b"ns:item:") + k[:6] for i, k in enumerate(base)]
        elif shape == "one_prefix":
            keys = [b"default:" + k for k in base]
        else:
            keys = base
        if shape == "sorted":
            keys = sorted(keys)
        vals = [bytes(rng.integers(0, 256, int(rng.integers(0, 30)), dtype=np.uint8)) for _ in keys]
        (ko, kd), (vo, vd) = _dev_batches(keys, vals)
        kb = gpu.KeyBatch(n=len(keys), data=kd, offsets=ko)
        vb = gpu.KeyBatch(n=len(vals), data=vd, offsets=vo)
        made.append(gpu.sstable_create((kb, vb), m=1 << 16, stream=st, wait=False))
        want.append((keys, vals))
    for (t, bloom, zone), (keys, vals) in zip(made, want):
        assert zone is None
        t.wait()
        assert t.data() == oracle.sstable_create(list(zip(keys, vals)))
        assert (t._zone(0), t._zone(1)) == (min(keys), max(keys))
        o = oracle.OracleFilter(1 << 16)
        for k in keys:
            o.insert(k)
        assert np.array_equal(bloom.bools(), o.bools())
        assert t.nlines == len(keys)


def test_create_bounded_refuses_a_batch_past_its_bounds(gpu):
    """cb_sstable_create_bounded sizes the file from the caller's byte
    bounds; a batch whose offsets go past them writes nothing and its table
    reports CB_EINVAL when finalised (no write past the buffer)."""
    import ctypes
    from lsmt_amd import _lib
    keys = [b"k%05d" % i for i in range(5000)]
    vals = [b"v" * 20 for _ in keys]
    (ko, kd), (vo, vd) = _dev_batches(keys, vals)
    L = _lib.load()
    th, fh = ctypes.c_void_p(), ctypes.c_void_p()
    rc = L.cb_sstable_create_bounded(kd.data_ptr(), ko.data_ptr(), 100, vd.data_ptr(), vo.data_ptr(),
                                     int(vd.numel()), len(keys), 1024, 0, None, ctypes.byref(th), ctypes.byref(fh))
    assert rc == 0
    assert L.cb_table_wait(th) == _lib.CB_EINVAL
    assert L.cb_table_wait(th) == _lib.CB_EINVAL  # sticky
    L.cb_table_destroy(th)
    L.cb_filter_destroy(fh)


def test_create_bounded_host_bytes_device_offsets(gpu):
    """Host key (or value) bytes with device offsets: the bytes are staged into
    a block of exactly the declared bounds, so offsets past them are refused
    by the call itself (CB_EINVAL, nothing enqueued, no table or filter
    returned), and a batch within them builds the reference's file and filter
    (the kernels used to read past the staged block)."""
    import ctypes
    from lsmt_amd import _lib
    keys = [b"h%05d" % i for i in range(3000)]
    vals = [b"w" * 12 for _ in keys]
    (ko, kd), (vo, vd) = _dev_batches(keys, vals)
    kh = kd.cpu().numpy()  # the same bytes in (pageable) host memory
    vh = vd.cpu().numpy()
    L = _lib.load()
    for kb, vb in ((kh, vd), (kd, vh)):  # host keys / host values, device offsets for both
        th, fh = ctypes.c_void_p(), ctypes.c_void_p()
        kp = kb.ctypes.data if isinstance(kb, np.ndarray) else kb.data_ptr()
        vp = vb.ctypes.data if isinstance(vb, np.ndarray) else vb.data_ptr()
        short_k = 100 if isinstance(kb, np.ndarray) else int(kd.numel())
        short_v = 100 if isinstance(vb, np.ndarray) else int(vd.numel())
        rc = L.cb_sstable_create_bounded(kp, ko.data_ptr(), short_k, vp, vo.data_ptr(), short_v, len(keys), 1024, 0,
                                         None, ctypes.byref(th), ctypes.byref(fh))
        assert rc == _lib.CB_EINVAL and not th.value and not fh.value
        rc = L.cb_sstable_create_bounded(kp, ko.data_ptr(), int(kd.numel()), vp, vo.data_ptr(), int(vd.numel()),
                                         len(keys), 1024, 0, None, ctypes.byref(th), ctypes.byref(fh))
        assert rc == 0 and L.cb_table_wait(th) == 0
        n = ctypes.c_uint64()
        dp = ctypes.c_void_p()
        assert L.cb_table_data(th, ctypes.byref(dp), ctypes.byref(n)) == 0
        buf = np.zeros(n.value, np.uint8)
        assert L.cb_table_copy(th, 0, n.value, buf.ctypes.data) == 0
        assert buf.tobytes() == oracle.sstable_create(list(zip(keys, vals)))
        o = oracle.OracleFilter(1024)
        for k in keys:
            o.insert(k)
        got = np.zeros(1024, np.uint8)
        assert L.cb_filter_export_bools(fh, got.ctypes.data, None) == 0
        assert np.array_equal(got, o.bools())
        L.cb_table_destroy(th)
        L.cb_filter_destroy(fh)


def test_create_pending_table_destroyed_unread(gpu):
    """A table destroyed before anything finalised it waits for its own work
    first (no buffer is reused under a running kernel)."""
    keys = [bytes(x) for x in workload.key_range(9700, 200_000)]
    vals = [b"x" * 8] * len(keys)
    (ko, kd), (vo, vd) = _dev_batches(keys, vals)
    for _ in range(3):
        t, b, _ = gpu.sstable_create((gpu.KeyBatch(n=len(keys), data=kd, offsets=ko),
                                      gpu.KeyBatch(n=len(vals), data=vd, offsets=vo)), m=1 << 20, wait=False)
        t.close()
        b.close()
    t, _, zone = gpu.sstable_create(list(zip(keys[:1000], vals[:1000])))
    assert t.data() == oracle.sstable_create(list(zip(keys[:1000], vals[:1000])))
