"""GPU parity for SURVEY.md §8f row 3: SSTable data files in HBM — the line
index, SsTable::binary_search for key batches, base64 decoding, and
Database::get's newest-first walk gated by the FilterSet probe. Exact against
the golden fixtures and the C oracle.

Reference: src/sstable.rs:57-72 (file format), 133-153 (get), 161-179
(binary_search), src/lib.rs:128-134 (newest-first walk).
"""
import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu


def var(keys):
    offs = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=offs[1:])
    data = np.frombuffer(b"".join(keys), np.uint8).copy() if offs[-1] else np.zeros(1, np.uint8)
    return data, offs


def oracle_lines(data: bytes):
    t = oracle.OracleTable(data)
    n = t.nlines
    st = np.ctypeslib.as_array(t._t.start, shape=(n,)).copy() if n else np.zeros(0, np.uint64)
    en = np.ctypeslib.as_array(t._t.end, shape=(n,)).copy() if n else np.zeros(0, np.uint64)
    return t, st, en


def check_index(gpu, data: bytes):
    t = gpu.Table(data)
    ot, st, en = oracle_lines(data)
    assert t.nlines == ot.nlines
    s, kl, ll = t.lines()
    assert np.array_equal(s, st)
    assert np.array_equal(ll.astype(np.uint64), en - st)
    raw = np.frombuffer(data, np.uint8)
    for i in range(0, ot.nlines, max(1, ot.nlines // 500)):
        line = raw[st[i]:en[i]]
        tabs = np.flatnonzero(line == 9)
        assert kl[i] == (tabs[0] if len(tabs) else 0xFFFFFFFF)
    return t, ot


def test_search_golden(gpu, golden):
    g = golden["sstable"]
    probes = [bytes.fromhex(p) for p in g["probes_hex"]]
    d, o = var(probes)
    kb = gpu.KeyBatch(n=len(probes), data=d, offsets=o)
    for name, hexdata in g["files_hex"].items():
        t, _ = check_index(gpu, bytes.fromhex(hexdata))
        lines = t.search(kb)
        assert list(lines) == [e["line"] for e in g["search"][name]], name


def test_get_many_golden(gpu, golden):
    g = golden["sstable"]
    probes = [bytes.fromhex(p) for p in g["probes_hex"]]
    d, o = var(probes)
    tables = [gpu.Table(bytes.fromhex(h)) for h in g["get_tables_hex"]]
    which, voff, vals = gpu.get_many(tables, gpu.KeyBatch(n=len(probes), data=d, offsets=o))
    for k, exp in enumerate(g["get"]):
        assert which[k] == exp["which"], probes[k]
        if exp["which"] >= 0:
            assert vals[voff[k]:voff[k + 1]].hex() == exp["value_hex"], probes[k]
        else:
            assert voff[k] == voff[k + 1]


@pytest.mark.parametrize("seed", [1, 2])
def test_index_random_bytes(gpu, seed):
    # dense '\n' / '\t' noise: empty lines, lines without TABs, chunk and
    # slice boundaries everywhere; also a file without a final newline
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"\n\n\t abc", np.uint8)
    for n in (1, 15, 16, 17, 4095, 4096, 4097, 300_001):
        data = rng.choice(alpha, n).tobytes()
        check_index(gpu, data)
    long_line = b"x" * 100_000 + b"\tQQ==\n" + b"y\n"
    check_index(gpu, long_line)


def test_search_random_files_vs_oracle(gpu):
    rng = np.random.default_rng(5)
    for n in (1, 2, 3, 16, 17, 256, 257, 1000, 4097, 70_001):  # fence levels L = 0..4
        keys = workload.key_range(900 + n, n)
        data = workload.sstable_bytes(keys, workload.table_value(keys, 3)).tobytes()
        t = gpu.Table(data)
        assert t.well_formed
        ot = oracle.OracleTable(data)
        look = np.concatenate([keys[rng.integers(0, n, 2000)], workload.key_range(77, 2000)])
        got = t.search(look)
        exp = [ot.search(bytes(k))[0] for k in look]
        assert list(got) == exp
        gpu.Table.force_exact(True)
        try:
            te = gpu.Table(data)
        finally:
            gpu.Table.force_exact(False)
        assert not te.well_formed and list(te.search(look)) == exp
        assert (got[:2000] >= 0).all() and (got[2000:] < 0).all()
    # ragged keys against a file with unsorted and TAB-less lines
    vk = [bytes(rng.integers(97, 100, rng.integers(0, 4), dtype=np.uint8)) for _ in range(3000)]
    lines = b"".join(k + (b"\tQQ==\n" if i % 7 else b"\n") for i, k in enumerate(sorted(set(vk))))
    t, ot = gpu.Table(lines), oracle.OracleTable(lines)
    assert not t.well_formed  # TAB-less lines: the exact trajectory
    d, o = var(vk)
    got = t.search(gpu.KeyBatch(n=len(vk), data=d, offsets=o))
    assert list(got) == [ot.search(k)[0] for k in vk]


def test_get_many_gated_vs_oracle(gpu):
    # 8 tables (newest first) over one key space; overlapping keys get newer
    # values; the FilterSet's gated probe decides which tables are searched
    m = 1 << 20
    nt = 8
    per = [workload.key_range(1200 + (t % 5), 40_000 + 1000 * t) for t in range(nt)]
    files = [workload.sstable_bytes(k, workload.table_value(k, 100 + t)) for t, k in enumerate(per)]
    tables = [gpu.Table(f) for f in files]
    otables = [oracle.OracleTable(f.tobytes()) for f in files]
    filters = []
    for k in per:
        b = gpu.BloomFilter(m)
        b.insert_batch(k)
        filters.append(b)
    s = gpu.FilterSet.from_filters(filters)
    for i, k in enumerate(per):
        s.zone_from_keys(i, k)
    look = np.concatenate([per[3][:30_000], per[7][-20_000:], workload.key_range(4321, 50_000)])
    look = look[np.random.default_rng(2).permutation(len(look))]
    hits = s.probe(look, gated=True)
    which, voff, vals = gpu.get_many(tables, look, hits=hits)
    d = np.ascontiguousarray(look.reshape(-1))
    offs = np.arange(0, 16 * (len(look) + 1), 16, dtype=np.uint64)
    ow, ovoff, ovals = oracle.get_many(otables, hits, d, offs)
    assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals
    # the exact-trajectory search gives the same answers on these files
    gpu.Table.force_exact(True)
    try:
        exact = [gpu.Table(f) for f in files]
    finally:
        gpu.Table.force_exact(False)
    we, voe, valse = gpu.get_many(exact, look, hits=hits)
    assert np.array_equal(we, ow) and valse == ovals
    # ungated = the same answers (the gate has no false negatives)
    w2, v2, vals2 = gpu.get_many(tables, look)
    assert np.array_equal(w2, ow) and vals2 == ovals
    # the value of a found key is table_value(key, 100 + table)
    k0 = int(np.flatnonzero(which >= 0)[0])
    t0 = int(which[k0])
    assert vals[voff[k0]:voff[k0 + 1]] == workload.table_value(look[k0:k0 + 1], 100 + t0).tobytes()
    # hit rows permuted: table t reads row rows[t]
    rows = np.arange(nt)[::-1].copy()
    w3, _, vals3 = gpu.get_many(tables, look, hits=hits[rows].copy(), hit_rows=rows)
    assert np.array_equal(w3, ow) and vals3 == ovals


def _fused_case(gpu, m, nt, width, seed):
    """nt tables (newest first) of overlapping key ranges, their filters in a
    FilterSet of `width` slots at a permuted slot each, zones on every other
    table only (the rest accept every key)."""
    per = [workload.key_range(1300 + (t % 3), 20_000 + 700 * t) for t in range(nt)]
    files = [workload.sstable_bytes(k, workload.table_value(k, 200 + t)) for t, k in enumerate(per)]
    tables = [gpu.Table(f) for f in files]
    otables = [oracle.OracleTable(f.tobytes()) for f in files]
    slots = np.random.default_rng(seed).permutation(width)[:nt].astype(np.uint32)
    s = gpu.FilterSet(m, width=width)
    for t, k in enumerate(per):
        b = gpu.BloomFilter(m)
        b.insert_batch(k)
        s.assign(int(slots[t]), b)
        if t % 2 == 0:
            s.zone_from_keys(int(slots[t]), k)
    look = np.concatenate([per[1][:9_000], per[nt - 1][-6_000:], workload.key_range(4322, 15_000)])
    look = look[np.random.default_rng(seed + 1).permutation(len(look))]
    return tables, otables, slots, s, look


@pytest.mark.parametrize("m,nt,width", [(1 << 20, 8, 32), (1_000_003, 5, 64), (1 << 20, 64, 64)])
def test_set_get_many_vs_oracle(gpu, m, nt, width):
    """cb_set_get_many_*: the zone + Bloom gate computed inside the search
    kernel gives exactly what FilterSet.probe(gated=True) + get_many gives,
    and both equal the oracle's walk over those gate bits — for 16-byte keys,
    ragged keys, permuted slots, width 32 and 64 and a non-power-of-two m."""
    tables, otables, slots, s, look = _fused_case(gpu, m, nt, width, seed=nt)
    full = s.probe(look, gated=True)
    hits = full[slots].copy()  # row t = table t's slot
    d = np.ascontiguousarray(look.reshape(-1))
    offs = np.arange(0, 16 * (len(look) + 1), 16, dtype=np.uint64)
    ow, ovoff, ovals = oracle.get_many(otables, hits, d, offs)
    which, voff, vals = gpu.get_many(tables, look, filterset=s, hit_rows=slots)
    assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals
    w2, v2, vals2 = gpu.get_many(tables, look, hits=full, hit_rows=slots)
    assert np.array_equal(w2, ow) and vals2 == ovals
    assert (which >= 0).sum() > 0 and (which < 0).sum() > 0
    # ragged keys (KEY_VAR): the same keys with some cut short, plus the empty key
    vk = [bytes(k) for k in look[:4000]] + [bytes(k[: i % 16]) for i, k in enumerate(look[4000:6000])] + [b""]
    dv, ov = var(vk)
    kb = gpu.KeyBatch(n=len(vk), data=dv, offsets=ov)
    vhits = s.probe(kb, gated=True)[slots].copy()
    ow, ovoff, ovals = oracle.get_many(otables, vhits, dv, ov)
    which, voff, vals = gpu.get_many(tables, kb, filterset=s, hit_rows=slots)
    assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals


def test_get_many_batches_of_changing_size(gpu):
    """Consecutive calls on one stream (reused workspaces: tile sums, value
    offsets) with batch sizes from 1 key to 70K keys, alternating the
    two-step and the fused form, each equal to the oracle."""
    per = [workload.key_range(1500 + t, 30_000) for t in range(3)]
    files = [workload.sstable_bytes(k, workload.table_value(k, 400 + t)) for t, k in enumerate(per)]
    tables = [gpu.Table(f) for f in files]
    otables = [oracle.OracleTable(f.tobytes()) for f in files]
    s = gpu.FilterSet(1 << 20)
    for t, k in enumerate(per):
        b = gpu.BloomFilter(1 << 20)
        b.insert_batch(k)
        s.assign(t, b)
    pool = np.concatenate([per[0], per[2], workload.key_range(4324, 30_000)])
    pool = pool[np.random.default_rng(5).permutation(len(pool))]
    for i, nk in enumerate([70_000, 300, 40_000, 1, 16_384, 16_385, 20_000]):
        look = np.ascontiguousarray(pool[:nk])
        d = np.ascontiguousarray(look.reshape(-1))
        offs = np.arange(0, 16 * (nk + 1), 16, dtype=np.uint64)
        ow, ovoff, ovals = oracle.get_many(otables, None, d, offs)
        which, voff, vals = gpu.get_many(tables, look, filterset=s) if i % 2 else gpu.get_many(tables, look)
        assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals, nk


def test_get_many_decode_scan_boundary(gpu):
    """Batches at the edge of the decode's own tile-sum scan (sstable.hip
    k_b64_decode<RAW>: up to 256K keys, 1024 tiles; one key more takes the
    k_tile_scan launch), on device and host outputs, each equal to the
    oracle, and a value buffer one byte short left untouched with the total
    still reported."""
    import torch
    per = [workload.key_range(1700 + t, 150_000) for t in range(2)]
    files = [workload.sstable_bytes(k, workload.table_value(k, 700 + t)) for t, k in enumerate(per)]
    tables = [gpu.Table(f) for f in files]
    otables = [oracle.OracleTable(f.tobytes()) for f in files]
    pool = np.concatenate([per[0], per[1], workload.key_range(4325, 40_000)])
    pool = pool[np.random.default_rng(9).permutation(len(pool))]
    for nk in (262_144, 262_145, 262_143, 255 * 256 + 1):
        look = np.ascontiguousarray(pool[:nk])
        d = np.ascontiguousarray(look.reshape(-1))
        offs = np.arange(0, 16 * (nk + 1), 16, dtype=np.uint64)
        ow, ovoff, ovals = oracle.get_many(otables, None, d, offs)
        which, voff, vals = gpu.get_many(tables, look)
        assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals, nk
        dw = torch.empty(nk, dtype=torch.int32, device="cuda")
        dv = torch.empty(nk + 1, dtype=torch.int64, device="cuda")
        short = torch.full((len(ovals) - 1,), 7, dtype=torch.uint8, device="cuda")
        dk = gpu.DeviceKeys(torch.from_numpy(look).cuda())
        _, _, total = gpu.get_many(tables, dk, out=(dw, dv, short))
        assert total == len(ovals) and bool((short == 7).all()), nk
        assert np.array_equal(dv.cpu().numpy().astype(np.uint64), ovoff), nk
        full = torch.empty(len(ovals), dtype=torch.uint8, device="cuda")
        _, _, total = gpu.get_many(tables, dk, out=(dw, dv, full))
        assert bytes(full.cpu().numpy()) == ovals and np.array_equal(dw.cpu().numpy(), ow), nk


def test_get_many_same_list_mutated_between_calls(gpu):
    """One table list passed batch after batch while it changes in place
    (get_many keeps its handle array per list object, lsmt_amd.bloom.
    _table_array): a table replaced by a new one, the list reordered, a table
    closed and its slot refilled, the list grown. Every call equals the
    oracle over the list as it is at that call."""
    per = [workload.key_range(1600 + t, 8_000) for t in range(4)]
    files = [workload.sstable_bytes(k, workload.table_value(k, 500 + t)) for t, k in enumerate(per)]
    pool = np.concatenate(per + [workload.key_range(4325, 8_000)])
    look = np.ascontiguousarray(pool[np.random.default_rng(6).permutation(len(pool))][:20_000])
    d = np.ascontiguousarray(look.reshape(-1))
    offs = np.arange(0, 16 * (len(look) + 1), 16, dtype=np.uint64)
    tables = [gpu.Table(f) for f in files[:3]]
    idx = [0, 1, 2]

    def check():
        ow, ovoff, ovals = oracle.get_many([oracle.OracleTable(files[i].tobytes()) for i in idx], None, d, offs)
        which, voff, vals = gpu.get_many(tables, look)
        assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals, idx

    check()
    check()  # the kept array
    tables[1], idx[1] = gpu.Table(files[3]), 3  # replaced
    check()
    tables.reverse()
    idx.reverse()
    check()
    tables[0].close()  # closed, then its slot refilled
    tables[0], idx[0] = gpu.Table(files[1]), 1
    check()
    tables.append(gpu.Table(files[0]))
    idx.append(0)
    check()


def test_set_get_many_long_keys_and_exact_tables(gpu):
    """The fused form over ragged keys of 0..40 bytes (the long-key compares
    past the 16-byte index words), with one table indexed for the exact
    reference trajectory and one holding undecodable values (Err falls
    through to older tables), zones on every slot; equal to the oracle's walk
    over FilterSet.probe(gated=True)'s bits."""
    import base64
    rng = np.random.default_rng(17)
    alpha = np.frombuffer(b"abcxyz019_:", np.uint8)
    def rkey():
        return bytes(alpha[rng.integers(0, len(alpha), rng.integers(0, 41))])
    nt = 4
    keysets = [sorted({rkey() for _ in range(6000)}) for _ in range(nt)]
    keysets[1] = sorted(set(keysets[1]) | set(keysets[0][::3]))  # shared keys: the newer table wins
    def line(k, t, i):
        v = bytes([(t * 31 + i + j) % 256 for j in range(i % 23)])
        enc = base64.b64encode(v) if not (t == 2 and i % 5 == 0) else b"!!!"  # undecodable
        return k + b"\t" + enc + b"\n"
    files = [b"".join(line(k, t, i) for i, k in enumerate(ks)) for t, ks in enumerate(keysets)]
    gpu.Table.force_exact(True)
    try:
        t3 = gpu.Table(files[3])
    finally:
        gpu.Table.force_exact(False)
    tables = [gpu.Table(f) for f in files[:3]] + [t3]
    otables = [oracle.OracleTable(f) for f in files]
    s = gpu.FilterSet(1 << 18)
    for t, ks in enumerate(keysets):
        d, o = var(ks)
        kb = gpu.KeyBatch(n=len(ks), data=d, offsets=o)
        b = gpu.BloomFilter(1 << 18)
        b.insert_batch(kb)
        s.assign(t, b)
        s.zone_from_keys(t, kb)
    look = [k for ks in keysets for k in ks[::7]] + [rkey() for _ in range(3000)]
    d, o = var(look)
    kb = gpu.KeyBatch(n=len(look), data=d, offsets=o)
    hits = s.probe(kb, gated=True)
    ow, ovoff, ovals = oracle.get_many(otables, hits, d, o)
    which, voff, vals = gpu.get_many(tables, kb, filterset=s)
    assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals
    assert (which == 3).any() and (which == 0).any() and (which < 0).any()


def test_set_get_many_async_device(gpu):
    """Device keys and outputs, total = NULL (enqueue only), slots = NULL
    (table t = slot t): val_off[n] carries the total; the answers equal the
    two-step form's."""
    import torch
    m, nt = 1 << 20, 6
    per = [workload.key_range(1400 + t, 30_000) for t in range(nt)]
    tables = [gpu.Table(workload.sstable_bytes(k, workload.table_value(k, 300 + t))) for t, k in enumerate(per)]
    filters = []
    for k in per:
        b = gpu.BloomFilter(m)
        b.insert_batch(k)
        filters.append(b)
    s = gpu.FilterSet.from_filters(filters)
    for t, k in enumerate(per):
        s.zone_from_keys(t, k)
    look = np.concatenate([per[2][:20_000], workload.key_range(4323, 12_000)])
    ew, evoff, evals = gpu.get_many(tables, look, hits=s.probe(look, gated=True))
    dk = torch.from_numpy(look).cuda()
    which = torch.zeros(len(look), dtype=torch.int32, device="cuda")
    voff = torch.zeros(len(look) + 1, dtype=torch.int64, device="cuda")
    vals = torch.zeros(len(evals) + 64, dtype=torch.uint8, device="cuda")
    assert gpu.get_many(tables, gpu.DeviceKeys(dk), filterset=s, out=(which, voff, vals), wait=False)[2] is None
    torch.cuda.synchronize()
    tot = int(voff[-1].item())
    assert tot == len(evals)
    assert np.array_equal(which.cpu().numpy(), ew)
    assert np.array_equal(voff.cpu().numpy().view(np.uint64), evoff)
    assert vals[:tot].cpu().numpy().tobytes() == evals
    with pytest.raises(ValueError):
        gpu.get_many(tables, look, hits=s.probe(look), filterset=s)


def test_well_formed_detection(gpu):
    # prefix-sharing keys (equal 8-byte prefixes, keys shorter than 8 bytes,
    # embedded NULs) in a well-formed file take the fast path and must agree
    # with the oracle
    keys = sorted({b"", b"a", b"a\x00", b"a\x00\x00", b"abcdefgh", b"abcdefgh\x00", b"abcdefghA",
                   b"abcdefghB", b"abcdefgi", b"b" * 20, b"b" * 21, b"\xff" * 9})
    data = b"".join(k + b"\tQQ==\n" for k in keys)
    t, ot = gpu.Table(data), oracle.OracleTable(data)
    assert t.well_formed
    probes = keys + [b"a\x00\x01", b"abcdefgh\x01", b"abcdefg", b"b" * 22, b"\xff" * 8, b"\xff" * 10, b"c"]
    d, o = var(probes)
    assert list(t.search(gpu.KeyBatch(n=len(probes), data=d, offsets=o))) == [ot.search(k)[0] for k in probes]
    # duplicates / unsorted / TAB-less are not well-formed
    for bad in (b"a\tQQ==\na\tQQ==\n", b"b\tQQ==\na\tQQ==\n", b"a\tQQ==\nb\n"):
        assert not gpu.Table(bad).well_formed


def test_search_device_resident(gpu):
    import torch
    keys = workload.key_range(31, 50_000)
    data = workload.sstable_bytes(keys, workload.table_value(keys, 1))
    t = gpu.Table(torch.from_numpy(data).cuda())  # data already in HBM
    dk = torch.from_numpy(keys[::-1].copy()).cuda()
    out = torch.zeros(len(keys), dtype=torch.int64, device="cuda")
    t.search(gpu.DeviceKeys(dk), out=out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert (got >= 0).all()
    srt = workload.sort_keys16(keys)
    assert np.array_equal(srt[got], keys[::-1])


def test_get_many_device_out_cap(gpu):
    # device output buffers: one pass; a value buffer smaller than the total is
    # left untouched and the total is still reported (then the caller retries)
    import torch
    keys = [b"k%05d" % i for i in range(3000)]
    vals = [bytes([i % 251]) * (i % 37) for i in range(3000)]
    t, _, _ = gpu.sstable_create(list(zip(keys, vals)))
    look = keys[::3] + [b"absent", b"k99999"]
    d = np.frombuffer(b"".join(look), np.uint8)
    offs = np.zeros(len(look) + 1, np.uint64)
    np.cumsum([len(k) for k in look], out=offs[1:])
    kb = gpu.KeyBatch(n=len(look), data=d, offsets=offs)
    want = b"".join(vals[::3])
    which = torch.empty(len(look), dtype=torch.int32, device="cuda")
    voff = torch.empty(len(look) + 1, dtype=torch.int64, device="cuda")
    small = torch.full((len(want) - 1,), 7, dtype=torch.uint8, device="cuda")
    _, _, total = gpu.get_many([t], kb, out=(which, voff, small))
    assert total == len(want)
    assert bool((small == 7).all())
    big = torch.full((len(want) + 64,), 7, dtype=torch.uint8, device="cuda")
    _, _, total = gpu.get_many([t], kb, out=(which, voff, big))
    assert total == len(want)
    assert bytes(big[:total].cpu().numpy()) == want and bool((big[total:] == 7).all())
    w = which.cpu().numpy()
    assert (w[:-2] == 0).all() and (w[-2:] == -1).all()
    vo = voff.cpu().numpy()
    assert vo[-1] == total and vo[-2] == vo[-3] == total


def test_get_many_value_lengths(gpu):
    """Decoded values of every length 0..40 bytes at every alignment (the
    one-wait path for <= 18-byte values and the 8-char loop above it), against
    Python's base64 on the same lines (src/sstable.rs:147-153)."""
    import base64

    rng = np.random.default_rng(11)
    n = 4000
    keys = sorted({bytes(rng.integers(97, 123, rng.integers(1, 24), dtype=np.uint8)) for _ in range(n)})
    vals = [bytes(rng.integers(0, 256, i % 41, dtype=np.uint8)) for i in range(len(keys))]
    data = b"".join(k + b"\t" + base64.b64encode(v) + b"\n" for k, v in zip(keys, vals))
    t = gpu.Table(data)
    look = list(keys) + [b"zzzz-absent", b""]
    d, o = var(look)
    which, voff, got = gpu.get_many([t], gpu.KeyBatch(n=len(look), data=d, offsets=o))
    for i, k in enumerate(look):
        if i < len(keys):
            assert which[i] == 0 and got[voff[i]:voff[i + 1]] == vals[i], k
        else:
            assert which[i] < 0 and voff[i] == voff[i + 1]


def test_search_shared_prefixes(gpu):
    """Keys that share their first 8+ bytes ('user0000...'): the fast search
    resolves them through the records (galloping over the equal-prefix run,
    src/sstable.rs:161-179's answer either way), for runs of 1 to 200k lines,
    keys of 8 to 40 bytes, and probes between, before, after and equal to a
    prefix of the lines' keys."""
    rng = np.random.default_rng(11)
    keys = set()
    keys.update(b"user0000" + b"%09d" % i for i in range(0, 400_000, 2))       # a 200k-line run, 17-B keys
    keys.update(b"acct%04d" % g + b"%06x" % j for g in range(40) for j in range(g * g + 1))  # runs of 1..1522
    keys.update(b"k" * 8 + bytes(rng.integers(97, 123, rng.integers(0, 33), dtype=np.uint8)) for _ in range(3000))
    keys.update(b"zz%06d" % i for i in range(5000))                             # exactly 8 bytes
    keys = sorted(keys)
    data = oracle.sstable_create([(k, b"v%d" % i) for i, k in enumerate(keys)])
    t = gpu.Table(data)
    assert t.well_formed
    ot = oracle.OracleTable(data)
    present = [keys[i] for i in rng.integers(0, len(keys), 6000)]
    absent = ([b"user0000" + b"%09d" % i for i in range(1, 40_000, 37)] +          # odd: between lines
              [b"user0000", b"user000", b"user00000", b"acct0003", b"a", b"", b"zz", b"zzz", b"\xff" * 20] +
              [k + b"\x00" for k in present[:500]] + [k[:-1] for k in present[:500] if len(k) > 8])
    look = present + absent
    d, o = var(look)
    got = t.search(gpu.KeyBatch(n=len(look), data=d, offsets=o))
    exp = [ot.search(k)[0] for k in look]
    assert list(got) == exp
    assert (np.array(exp[:len(present)]) >= 0).all()
    # and through get_many (values decode from the found lines)
    which, voff, vals = gpu.get_many([t], gpu.KeyBatch(n=len(look), data=d, offsets=o))
    ow, ovoff, ovals = oracle.get_many([ot], None, d, o)
    assert np.array_equal(which, ow) and vals == ovals


def _check_rebuild(gpu, data: bytes, m: int):
    t = gpu.Table(data)
    ot = oracle.OracleTable(data)
    try:
        of, oz = ot.rebuild(m)
    except ValueError:
        with pytest.raises(UnicodeDecodeError):
            t.rebuild(m)
        return None
    f, z = t.rebuild(m)
    assert f.m == m
    assert np.array_equal(f.bools(), of.bools())
    assert (z.min, z.max) == oz.bounds
    return f, z


@pytest.mark.parametrize("m", [1024, 100003, 1 << 22])
def test_table_rebuild_vs_oracle(gpu, m):
    """SsTable::load without a usable .meta (src/sstable.rs:109-120): the
    filter and zone map rebuilt on the device from the data file equal the
    oracle's restatement: well-formed files, files with TAB-less and empty
    lines, unsorted files, empty keys, multi-byte UTF-8 keys, and files whose
    keys are not UTF-8 (the load fails)."""
    rng = np.random.default_rng(m % 97)
    keys = workload.key_range(3100, 50_000)
    _check_rebuild(gpu, workload.sstable_bytes(keys, workload.table_value(keys, 1)).tobytes(), m)
    # unsorted, TAB-less and empty lines, empty keys, tabs inside values
    lines = [b"%s\tQQ==" % bytes(k) for k in keys[:3000]][::-1]
    lines += [b"no separator here", b"", b"\tempty-key", b"k\twith\ttabs", b"\t", b"zz\t"]
    rng.shuffle(lines)
    _check_rebuild(gpu, b"\n".join(lines) + b"\n", m)
    # multi-byte UTF-8 keys (2-, 3- and 4-byte sequences) and a file with no final newline
    uk = ["é", "日本", "𝄞x", "a߿", "퟿", "\U0010ffff"]
    _check_rebuild(gpu, b"\n".join(k.encode() + b"\tQQ==" for k in uk), m)
    # no TAB anywhere, and an empty file: an empty filter, no zone bounds
    r = _check_rebuild(gpu, b"just\nlines\n", m)
    assert r[1].min is None and not r[0].bools().any()
    # keys that are not UTF-8: overlong, surrogate, > U+10FFFF, truncated, bare continuation
    for bad in (b"\xc0\xaf", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xe6\x97", b"\x80", b"ok\xff"):
        data = b"a\tQQ==\n" + bad + b"\tQQ==\nno-tab-\xff-line\n"
        assert _check_rebuild(gpu, data, m) is None, bad
    # invalid bytes on a TAB-less line or after the TAB do not matter
    assert _check_rebuild(gpu, b"\xff\xfe\nk\t\xff\n", m) is not None


def _keys_hi(hi: np.ndarray, seed: int) -> np.ndarray:
    """16-byte keys whose first 8 bytes are hi (big-endian), the rest random."""
    lo = np.random.default_rng(seed).integers(0, 1 << 63, len(hi), dtype=np.uint64)
    k = np.empty((len(hi), 2), dtype=">u8")
    k[:, 0], k[:, 1] = hi, lo
    b = k.view(np.uint8).reshape(-1, 16).copy()
    b[(b == 9) | (b == 10)] = 11  # no TAB / newline inside a key
    return np.unique(b, axis=0)


@pytest.mark.parametrize("shape", ["uniform", "shared20", "shared60", "clustered", "equal", "hex", "rare", "text"])
def test_search_directory_vs_oracle(gpu, shape):
    """The byte-rank directory (sstable.hpp DirMap / dir_bucket / dir_start)
    under prefix distributions that move its digits: uniform prefixes, 20 and
    60 shared leading bits, a clustered set with long runs of empty buckets,
    one equal prefix, 16-hex-char text keys (the bench's), hex keys with a few
    rare bytes the 8192-line sample misses ('rare': their digits are forced,
    sstable.hpp), and 'user'+digits keys. Probes: present keys, absent keys,
    prefixes at bucket edges, outside the key range on both sides, and keys
    with a byte just outside the alphabet at each position. t.search,
    get_many (the staged kernel, <= 64 tables) and the exact trajectory agree
    with the oracle."""
    rng = np.random.default_rng({"uniform": 1, "shared20": 2, "shared60": 3, "clustered": 4, "equal": 5,
                                 "hex": 6, "rare": 7, "text": 8}[shape])
    for n in (255, 256, 257, 5000, 70_001):
        keys = _dir_keys(shape, n, rng)
        data = workload.sstable_bytes(keys, workload.table_value(keys, 2)).tobytes()
        ot = oracle.OracleTable(data)
        _check_dir_table(gpu, gpu.Table(data), ot, keys, rng, n)
        # the same file from the device flush (its k_format writes the
        # directory), from sorted and from shuffled entries
        ents = [(bytes(k), bytes(v)) for k, v in zip(keys, workload.table_value(keys, 2))]
        for order in (None, rng.permutation(len(ents))):
            t2, _, _ = gpu.sstable_create(ents if order is None else [ents[i] for i in order])
            _check_dir_table(gpu, t2, ot, keys, rng, n)


def _text_keys(shape, n, rng):
    if shape == "hex":
        return workload.sort_keys16(workload.key_range(int(rng.integers(1, 1 << 20)), n))
    if shape == "rare":
        k = workload.key_range(int(rng.integers(1, 1 << 20)), n).copy()
        pick = rng.choice(n, max(1, n // 300), replace=False)
        k[pick, rng.integers(0, 8, len(pick))] = rng.choice(np.frombuffer(b"GHXYZ~!%" + bytes(range(0xC0, 0xC8)),
                                                                          np.uint8), len(pick))
        return np.unique(k, axis=0)
    d = rng.integers(0, 10, (n, 12), dtype=np.uint8) + ord("0")  # "user" + 12 digits
    k = np.concatenate([np.frombuffer(b"user", np.uint8)[None, :].repeat(n, 0), d], 1)
    return np.unique(k, axis=0)


def _dir_keys(shape, n, rng):
    if shape in ("hex", "rare", "text"):
        return _text_keys(shape, n, rng)
    if shape == "uniform":
        hi = rng.integers(0, 1 << 64, n, dtype=np.uint64)
    elif shape == "shared20":
        hi = (np.uint64(0xABCDE) << np.uint64(44)) | rng.integers(0, 1 << 44, n, dtype=np.uint64)
    elif shape == "shared60":
        hi = (np.uint64(0x123456789ABCDEF) << np.uint64(4)) | rng.integers(0, 16, n, dtype=np.uint64)
    elif shape == "clustered":
        a = rng.integers(0, 1 << 40, n // 2, dtype=np.uint64) + np.uint64(1 << 62)
        b = rng.integers(0, 1 << 64, n - n // 2, dtype=np.uint64)
        hi = np.concatenate([a, b])
    else:
        hi = np.full(n, 0x7573657230303030, dtype=np.uint64)
    return _keys_hi(hi, n)


def _check_dir_table(gpu, t, ot, keys, rng, n):
    assert t.well_formed
    h = keys[:, :8].copy().view(">u8").reshape(-1).astype(np.uint64)
    edges = []
    for x in h[rng.integers(0, len(h), 200)]:
        for bits in (4, 12, 20, 40):  # bucket-edge prefixes around present keys
            m = np.uint64((1 << bits) - 1)
            edges += [x & ~m, x | m]
    edges += [0, (1 << 64) - 1, int(h.min()) - 1 if h.min() else 0, int(h.max()) + 1 if h.max() < (1 << 64) - 1 else 0]
    eh = np.array(edges, dtype=np.uint64)
    absent = _keys_hi(np.concatenate([eh, rng.integers(0, 1 << 64, 2000, dtype=np.uint64)]), 7)
    # present keys with one prefix byte moved just outside / inside the
    # alphabet at each position (bytes the directory's sample never saw)
    near = keys[rng.integers(0, len(keys), 400)].copy()
    pos = rng.integers(0, 8, len(near))
    near[np.arange(len(near)), pos] = rng.choice(np.frombuffer(b"/:@`gG\x00\xff\x7f0af9", np.uint8), len(near))
    look = np.concatenate([keys[rng.integers(0, len(keys), 3000)], absent, near, keys[:1], keys[-1:]])
    exp = [ot.search(bytes(k))[0] for k in look]
    assert list(t.search(look)) == exp, n
    which, voff, vals = gpu.get_many([t], look)
    d = np.ascontiguousarray(look.reshape(-1))
    offs = np.arange(0, 16 * (len(look) + 1), 16, dtype=np.uint64)
    ow, ovoff, ovals = oracle.get_many([ot], None, d, offs)
    assert np.array_equal(which, ow) and vals == ovals, n


def test_get_many_past_64_tables_vs_oracle(gpu):
    """More than 64 tables: get_many's lane-per-search form (tables past the
    first 64 read their views from HBM, the first 64 from LDS with their
    directories), gated and ungated, against the oracle."""
    rng = np.random.default_rng(21)
    nt = 70
    per = [workload.key_range(3000 + t, 300 + 40 * t) for t in range(nt)]
    files = [workload.sstable_bytes(k, workload.table_value(k, t)) for t, k in enumerate(per)]
    tables = [gpu.Table(f) for f in files]
    otables = [oracle.OracleTable(f.tobytes()) for f in files]
    look = np.concatenate([per[t][rng.integers(0, len(per[t]), 100)] for t in range(nt)] +
                          [workload.key_range(99, 3000)])
    look = look[rng.permutation(len(look))]
    d = np.ascontiguousarray(look.reshape(-1))
    offs = np.arange(0, 16 * (len(look) + 1), 16, dtype=np.uint64)
    ow, ovoff, ovals = oracle.get_many(otables, None, d, offs)
    which, voff, vals = gpu.get_many(tables, look)
    assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals
    assert (ow >= 0).sum() == 100 * nt and (ow >= 64).any()


def test_get_many_async_and_view_cache(gpu):
    """get_many(wait=False) (C ABI total = NULL): enqueue only, the total in
    val_off[n]; consecutive calls on one stream with different table lists and
    hit rows (the views / rows upload cache must refresh) and the same lists
    again all give the synchronous answers."""
    import torch
    rng = np.random.default_rng(8)
    per = [workload.key_range(5100 + t, 2000 + 700 * t) for t in range(5)]
    tables = [gpu.Table(workload.sstable_bytes(k, workload.table_value(k, t))) for t, k in enumerate(per)]
    look = np.concatenate([per[t][rng.integers(0, len(per[t]), 500)] for t in range(5)] +
                          [workload.key_range(42, 1000)])
    look = look[rng.permutation(len(look))]
    dk = gpu.DeviceKeys(torch.from_numpy(look.copy()).cuda())
    n = len(look)
    lists = [tables, tables[::-1], tables[1:4], tables]
    s = torch.cuda.Stream()
    outs = []
    for tl in lists:
        o = (torch.empty(n, dtype=torch.int32, device="cuda"), torch.empty(n + 1, dtype=torch.int64, device="cuda"),
             torch.empty(n * 16, dtype=torch.uint8, device="cuda"))
        assert gpu.get_many(tl, dk, out=o, stream=s, wait=False)[2] is None
        outs.append(o)
    s.synchronize()
    for tl, (w, vo, vals) in zip(lists, outs):
        ew, evo, evals = gpu.get_many(tl, look)
        tot = int(vo[n].item())
        assert np.array_equal(w.cpu().numpy(), ew) and tot == len(evals)
        assert np.array_equal(vo.cpu().numpy().astype(np.uint64), evo)
        assert bytes(vals[:tot].cpu().numpy()) == evals
    # hit rows change between calls on one stream
    hits = np.zeros((5, (n + 63) // 64), dtype=np.uint64)
    hits[0::2] = ~np.uint64(0)  # rows 0, 2, 4 admit every key, rows 1, 3 none
    hd = torch.from_numpy(hits.view(np.int64)).cuda()
    res = []
    for rows in (np.array([1, 2, 3, 4, 0]), np.arange(5)):
        o = (torch.empty(n, dtype=torch.int32, device="cuda"), torch.empty(n + 1, dtype=torch.int64, device="cuda"),
             torch.empty(n * 16, dtype=torch.uint8, device="cuda"))
        gpu.get_many(tables, dk, hits=hd, hit_rows=rows, out=o, stream=s, wait=False)
        res.append(o)
    s.synchronize()
    for rows, (w, _, _) in zip((np.array([1, 2, 3, 4, 0]), np.arange(5)), res):
        ew, _, _ = gpu.get_many(tables, look, hits=hits, hit_rows=rows)
        assert np.array_equal(w.cpu().numpy(), ew)
    assert not np.array_equal(res[0][0].cpu().numpy(), res[1][0].cpu().numpy())
    # host outputs are refused without a total
    with pytest.raises(Exception):
        gpu.get_many(tables, look, out=(np.zeros(n, np.int32), np.zeros(n + 1, np.uint64), np.zeros(16, np.uint8)),
                     wait=False)


def test_get_many_key_buckets(gpu):
    """The read path's key buckets (sstable.hpp, built by a table's first
    get_many): tables whose lines share 8-byte prefixes (many lines per
    prefix, so buckets overflow and prefixes collide), lines left out of the
    buckets (a 5000-byte key, values decoding to more than 4095 bytes, an
    undecodable value), tables of 1 and 3 lines; the first call (buckets built
    on its stream), a second one, and one on another stream right after the
    first (buckets maybe not yet usable there) all equal the oracle."""
    import base64
    import torch
    rng = np.random.default_rng(23)
    shared = sorted({b"user0000" + bytes(rng.integers(48, 58, 6, dtype=np.uint8)) for _ in range(3000)})
    plain = [bytes(k) for k in workload.key_range(2400, 20_000)]
    def lines(keys, t):
        out = []
        for i, k in enumerate(keys):
            if t == 1 and i % 97 == 0:
                v = base64.b64encode(bytes(5000))  # decodes to 5000 bytes: left out of the buckets
            elif t == 1 and i % 89 == 0:
                v = b"!!"  # undecodable
            else:
                v = base64.b64encode(bytes([(i + t) % 256] * (i % 20)))
            out.append(k + b"\t" + v + b"\n")
        return b"".join(out)
    big = sorted(plain[:5000] + [b"zz" + b"k" * 4998])  # one 5000-byte key
    keysets = [shared, sorted(plain), big, [b"aaa-single"], [b"mmm1", b"mmm2", b"mmm3"]]
    files = [lines(ks, t) for t, ks in enumerate(keysets)]
    tables = [gpu.Table(f) for f in files]
    assert all(t.well_formed for t in tables)
    otables = [oracle.OracleTable(f) for f in files]
    look = ([k for ks in keysets for k in ks[::3]] + [b"user0000" + bytes(rng.integers(48, 58, 6, dtype=np.uint8))
                                                      for _ in range(2000)] + [bytes(k) for k in workload.key_range(2401, 3000)])
    d, o = var(look)
    kb = gpu.KeyBatch(n=len(look), data=d, offsets=o)
    ow, ovoff, ovals = oracle.get_many(otables, None, d, o)
    dev = torch.device("cuda", 0)
    other = torch.cuda.Stream(device=dev)
    for i in range(3):
        which, voff, vals = gpu.get_many(tables, kb, stream=other if i == 1 else None)
        assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals, i
    assert (which >= 0).sum() > 0.3 * len(look) and all((which == t).any() for t in range(5))


def test_get_many_bucket_budget_and_cross_stream_waits(gpu):
    """cb_table_bucket_limit: tables read while the limit is 0 (or below their
    buckets' size) are searched without key buckets, with the reference's
    answers; later tables get them again at the default. Reads on several
    streams right after a table's first read enqueue a wait for its bucket
    build (no stream-handle identity), and every answer equals the
    oracle's."""
    import torch
    keys = [bytes(k) for k in workload.key_range(2500, 30_000)]
    data = b"".join(k + b"\t" + base64_of(i) + b"\n" for i, k in enumerate(sorted(keys)))
    look = keys[::5] + [bytes(k) for k in workload.key_range(2501, 4000)]
    d, o = var(look)
    kb = gpu.KeyBatch(n=len(look), data=d, offsets=o)
    ow, ovoff, ovals = oracle.get_many([oracle.OracleTable(data)], None, d, o)
    try:
        gpu.Table.bucket_limit(0)
        t0 = gpu.Table(data)
        which, voff, vals = gpu.get_many([t0], kb)
        assert np.array_equal(which, ow) and np.array_equal(voff, ovoff) and vals == ovals
        gpu.Table.bucket_limit(1024)  # smaller than this table's 2^15 x 136 B
        t1 = gpu.Table(data)
        which, voff, vals = gpu.get_many([t1], kb)
        assert np.array_equal(which, ow) and vals == ovals
    finally:
        gpu.Table.bucket_limit(1 << 30)
    t2 = gpu.Table(data)
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(device=dev) for _ in range(4)]
    n = len(look)
    kd = gpu.KeyBatch(n=n, data=torch.from_numpy(d).to(dev), offsets=torch.from_numpy(o.view(np.int64)).to(dev))
    bufs = [(torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n + 1, dtype=torch.int64, device=dev),
             torch.empty(len(ovals) + 16, dtype=torch.uint8, device=dev)) for _ in streams]
    # enqueue-only reads on four streams, back to back: the first builds the
    # buckets on its stream, the other three enqueue waits for that build
    with torch.cuda.stream(streams[0]):
        torch.cuda._sleep(20_000_000)  # hold the building stream so the others queue behind its event
    for st, out in zip(streams, bufs):
        gpu.get_many([t2], kd, stream=st, out=out, wait=False)
    torch.cuda.synchronize()
    for which, voff, vals in bufs:
        tot = int(voff[n].item())
        assert np.array_equal(which.cpu().numpy(), ow)
        assert np.array_equal(voff.cpu().numpy().view(np.uint64), ovoff)
        assert bytes(vals[:tot].cpu().numpy()) == ovals


def base64_of(i):
    import base64
    return base64.b64encode(b"val%d" % i)
