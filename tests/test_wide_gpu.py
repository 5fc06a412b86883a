"""Wide filter sets (more than 64 SSTable filters in one set): the
reference's real read-path shape. Every table's filter is m = 1024
(/root/reference/src/sstable.rs:44,59) and the memtable flushes every 1024
inserts (src/lib.rs:72,105), so Database::get walks hundreds of tables
newest first (src/lib.rs:129-134), each behind SsTable::get's gate
zone_map.contains && bloom.may_contain (src/sstable.rs:138). Checked bit for
bit against the oracle: the hit rows of the plain and gated probe, and the
fused one-launch get_many over 300 auto-flush-sized tables with every table
-> slot mapping the kernel distinguishes (ascending, descending, scattered)."""
import numpy as np
import pytest

from lsmt_amd import workload
from oracle import oracle

pytestmark = pytest.mark.gpu


def _ragged(keys):
    offs = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=offs[1:])
    return np.frombuffer(b"".join(keys) or b"\0", np.uint8).copy(), offs


@pytest.fixture(scope="module")
def lsm300(gpu):
    """300 tables as 300 auto-flushes of 1024 entries would leave them: keys
    drawn from a shared pool (a key rewritten in a later flush lives in
    several tables, the newest value wins), values naming the table."""
    rng = np.random.default_rng(300)
    pool = workload.key_range(4242, 120_000)
    nt, per = 300, 1024
    tables, blooms, zones, entries = [], [], [], []
    for t in range(nt):  # t = age order: table 0 oldest
        idx = np.unique(rng.choice(len(pool), per, replace=False))
        ents = [(bytes(pool[i]), b"t%03d:%d" % (t, i)) for i in idx]
        tb, bloom, zone = gpu.sstable_create(ents, m=1024)
        tables.append(tb)
        blooms.append(bloom)
        zones.append(zone)
        entries.append(ents)
    present = pool[rng.integers(0, len(pool), 6000)]
    absent = workload.key_range(4343, 2000)
    look = np.concatenate([present, absent])[rng.permutation(8000)]
    return dict(tables=tables, blooms=blooms, zones=zones, entries=entries, look=look, pool=pool)


def _oracle_expect(d, order):
    """Oracle Database::get over tables in `order` (newest first): the gate
    rows (zone && bloom per table), then the newest-first walk."""
    look = d["look"]
    data, offs = np.ascontiguousarray(look.reshape(-1)), np.arange(0, 16 * (len(look) + 1), 16, dtype=np.uint64)
    ofs, ozs, ots = [], [], []
    for t in order:
        o = oracle.OracleFilter(1024)
        for k, _ in d["entries"][t]:
            o.insert(k)
        ofs.append(o)
        ozs.append(oracle.OracleZone(d["zones"][t].min, d["zones"][t].max))
        ots.append(oracle.OracleTable(d["tables"][t].data()))
    gate = oracle.probe_gated(ofs, ozs, data, offs)
    return oracle.get_many(ots, gate, data, offs)


@pytest.mark.parametrize("mapping", ["descending", "ascending", "scattered"])
def test_wide_get_many_300_tables(gpu, lsm300, mapping):
    d = lsm300
    nt = len(d["tables"])
    s = gpu.FilterSet(1024, width=320)
    rng = np.random.default_rng(7)
    if mapping == "descending":  # slot = age (Vec<SsTable> index), walked .rev(): the LSM's own order
        slot_of_age = np.arange(nt)
    elif mapping == "ascending":  # slot 0 holds the newest table
        slot_of_age = np.arange(nt)[::-1].copy()
    else:
        slot_of_age = rng.permutation(320)[:nt]
    for age in range(nt):
        s.assign(int(slot_of_age[age]), d["blooms"][age])
        s.set_zone(int(slot_of_age[age]), d["zones"][age])
    newest_first = list(range(nt))[::-1]
    tabs = [d["tables"][a] for a in newest_first]
    slots = slot_of_age[newest_first].astype(np.uint32)
    which, voff, vals = gpu.get_many(tabs, d["look"], filterset=s, hit_rows=slots)
    ow, ovoff, ovals = _oracle_expect(d, newest_first)
    assert np.array_equal(np.asarray(which), ow)
    assert np.array_equal(np.asarray(voff, dtype=np.uint64), ovoff) and vals == ovals
    assert (np.asarray(which) >= 0).sum() >= 5000  # most present keys live in some table (pool of 120K, 307K draws)


def test_wide_probe_rows_match_oracle(gpu, lsm300):
    """cb_set_probe on a wide set: [used][n/64] rows, plain and gated, against
    the oracle's may_contain and zone && may_contain per slot."""
    d = lsm300
    nt = len(d["tables"])
    s = gpu.FilterSet.from_filters(d["blooms"])
    assert s.width == 320 and s.used == nt
    look = d["look"]
    data, offs = np.ascontiguousarray(look.reshape(-1)), np.arange(0, 16 * (len(look) + 1), 16, dtype=np.uint64)
    ofs = []
    for t in range(nt):
        o = oracle.OracleFilter(1024)
        for k, _ in d["entries"][t]:
            o.insert(k)
        ofs.append(o)
    assert np.array_equal(s.probe(look), oracle.probe_fixed(ofs, look))
    for t in range(nt):
        s.set_zone(t, d["zones"][t])
    ozs = [oracle.OracleZone(z.min, z.max) for z in d["zones"]]
    assert np.array_equal(s.probe(look, gated=True), oracle.probe_gated(ofs, ozs, data, offs))
    # a reset slot (re-assigned filter) drops its zone: the gate accepts every key there again
    s.assign(5, d["blooms"][5])
    ozs[5] = None
    assert np.array_equal(s.probe(look, gated=True), oracle.probe_gated(ofs, ozs, data, offs))


@pytest.mark.parametrize("m,width,nf", [(1 << 20, 128, 70), (100003, 192, 130)])
def test_wide_ragged_keys_and_updates(gpu, m, width, nf):
    """Larger and non-power-of-two m, ragged keys (the product's "ns:pk|ck"
    strings), and every maintenance path: the one-launch build, the sparse OR
    into an empty slot, the dense rewrite of a used slot, a cleared slot."""
    rng = np.random.default_rng(m + nf)
    data, offs = workload.var_keys(rng, 30_000, max_len=40)
    keys = [data[offs[i]:offs[i + 1]].tobytes() for i in range(len(offs) - 1)]
    fs, ofs = [], []
    for f in range(nf):
        ks = [keys[i] for i in rng.integers(0, len(keys), 2000)]
        b = gpu.BloomFilter(m)
        kd, ko = _ragged(ks)
        b.insert_batch(gpu.KeyBatch(n=len(ks), data=kd, offsets=ko))
        o = oracle.OracleFilter(m)
        o.insert_var(kd, ko)
        fs.append(b)
        ofs.append(o)
    s = gpu.FilterSet.from_filters(fs[:-2], width=width)
    s.assign(nf - 2, fs[-2])           # empty slot: sparse OR
    s.assign(3, fs[-1])                # used slot: dense rewrite
    s.clear_slot(7)
    expect = [ofs[i] for i in range(nf - 1)]
    expect[3] = ofs[-1]
    expect[7] = oracle.OracleFilter(m)
    got = s.probe(gpu.KeyBatch(n=len(keys), data=data, offsets=offs))
    assert np.array_equal(got, oracle.probe_var(expect, data, offs))


def test_wide_screen_mixed_buckets_and_rebuilt_tables(gpu):
    """The wide walk's screen (sstable.hpp WideScreen: per bucket and
    fingerprint bin, one bit per slot that could still hold the key) against
    the oracle's walk: tables of two bucket counts (the screen speaks for the
    common one, the others always pass), tables whose keys share their first
    8 bytes (crowded buckets past four lines: no proof of absence), the same
    call repeated (the cached screen), and tables replaced by new ones (the
    screen is rebuilt from the new tables' ids, not their addresses)."""
    rng = np.random.default_rng(77)
    pool = workload.key_range(5151, 40_000)

    def make(t):
        if t % 17 == 5:  # crowded: 600 keys sharing the 8-byte prefix "crowded:"
            ks = [b"crowded:" + bytes(pool[i][:8]) for i in rng.choice(len(pool), 600, replace=False)]
        else:
            nk = 3000 if t % 11 == 3 else 1024  # 2^12 buckets for some tables, 2^10 for most
            ks = [bytes(pool[i]) for i in rng.choice(len(pool), nk, replace=False)]
        ks = sorted(set(ks))
        ents = [(k, b"v%03d:%s" % (t, k[-4:])) for k in ks]
        tb, bloom, zone = gpu.sstable_create(ents, m=1024)
        return tb, bloom, zone, ents

    nt = 130
    made = [make(t) for t in range(nt)]
    crowd = [b"crowded:" + bytes(pool[i][:8]) for i in rng.integers(0, len(pool), 1000)]
    look = np.concatenate([pool[rng.integers(0, len(pool), 5000)], workload.key_range(5252, 1000),
                           np.frombuffer(b"".join(crowd), np.uint8).reshape(-1, 16)])[rng.permutation(7000)]

    def expect():
        data, offs = np.ascontiguousarray(look.reshape(-1)), np.arange(0, 16 * (len(look) + 1), 16, dtype=np.uint64)
        ofs, ozs, ots = [], [], []
        for t in range(nt - 1, -1, -1):
            tb, _, zone, ents = made[t]
            o = oracle.OracleFilter(1024)
            for k, _ in ents:
                o.insert(k)
            ofs.append(o)
            ozs.append(oracle.OracleZone(zone.min, zone.max))
            ots.append(oracle.OracleTable(tb.data()))
        return oracle.get_many(ots, oracle.probe_gated(ofs, ozs, data, offs), data, offs)

    def run():
        s = gpu.FilterSet(1024, width=192)
        for t in range(nt):
            s.assign(t, made[t][1])
            s.set_zone(t, made[t][2])
        tabs = [made[t][0] for t in range(nt - 1, -1, -1)]
        slots = np.arange(nt, dtype=np.uint32)[::-1].copy()
        return gpu.get_many(tabs, look, filterset=s, hit_rows=slots)

    for _ in range(2):  # the second call reuses the stream's screen
        which, voff, vals = run()
        ow, ovoff, ovals = expect()
        assert np.array_equal(np.asarray(which), ow)
        assert np.array_equal(np.asarray(voff, dtype=np.uint64), ovoff) and vals == ovals
    for t in (0, 40, 77, 129):  # replaced tables: new content, possibly at the old addresses
        made[t] = None
    import gc
    gc.collect()
    for t in (0, 40, 77, 129):
        made[t] = make(t + 1000)
    which, voff, vals = run()
    ow, ovoff, ovals = expect()
    assert np.array_equal(np.asarray(which), ow)
    assert np.array_equal(np.asarray(voff, dtype=np.uint64), ovoff) and vals == ovals


@pytest.mark.parametrize("mapping", ["descending", "scattered"])
def test_wide_get_many_348_tables(gpu, lsm300, mapping):
    """Six groups of 64 with a partial last one: 348 tables (the 300 plus the
    48 oldest listed again, behind them, so absent keys walk them twice) in a
    384-slot set, checked against the oracle like the 300-table case."""
    d = lsm300
    ages = list(range(48)) + list(range(300))  # position = age order: the 48 re-listed ones are the oldest
    nt = len(ages)
    s = gpu.FilterSet(1024, width=384)
    slot_of_pos = np.arange(nt) if mapping == "descending" else np.random.default_rng(9).permutation(384)[:nt]
    for pos, age in enumerate(ages):
        s.assign(int(slot_of_pos[pos]), d["blooms"][age])
        s.set_zone(int(slot_of_pos[pos]), d["zones"][age])
    newest_first = list(range(nt))[::-1]
    tabs = [d["tables"][ages[p]] for p in newest_first]
    slots = slot_of_pos[newest_first].astype(np.uint32)
    which, voff, vals = gpu.get_many(tabs, d["look"], filterset=s, hit_rows=slots)
    ow, ovoff, ovals = _oracle_expect(d, [ages[p] for p in newest_first])
    assert np.array_equal(np.asarray(which), ow)
    assert np.array_equal(np.asarray(voff, dtype=np.uint64), ovoff) and vals == ovals
