/*
 * cassbloom.h — C ABI of the MI355X-native Bloom-filter path for the `cass`
 * LSM store (mweiden/lsmt). Drop-in for /root/reference/src/bloom.rs.
 *
 * Every entry point is plain C: opaque handles, pointers and sizes; no HIP,
 * torch or C++ types. Streams are passed as `void*` (a hipStream_t; NULL = the
 * device's null stream). Return value: CB_OK (0) or a negative CB_E* code;
 * cb_last_error() gives a thread-local message for the last failure.
 *
 * Bit layout of a device filter (the "packed" form): bit p of the reference's
 * Vec<bool> lives in 32-bit word p>>5 at bit p&31 (LSB-first), i.e. byte p>>3
 * bit p&7 — little-endian packbits(bitorder="little") of the bool array.
 *
 * Pointer residency: key, offset and hit buffers may be device memory
 * (hipMalloc / torch) or host memory (pageable or pinned). Device buffers are
 * used in place and the call is asynchronous on `stream`. Host buffers are
 * staged through library-owned device buffers and the call synchronises the
 * stream before returning, so host outputs are valid on return.
 *
 * Reference interface replaced by each entry point (file:line in
 * /root/reference):
 *   cb_filter_create        BloomFilter::new(size)               src/bloom.rs:17-21
 *   cb_filter_insert_*      BloomFilter::insert(&mut, &str)      src/bloom.rs:40-44
 *                           batched over SsTable::create's loop  src/sstable.rs:62-65
 *                           and SsTable::load's rebuild loop     src/sstable.rs:113-119
 *   cb_probe_*              BloomFilter::may_contain(&, &str)    src/bloom.rs:48-51
 *                           batched over Database::get's fan-out src/lib.rs:129-134
 *   cb_may_contain          BloomFilter::may_contain (one key)   src/bloom.rs:48-51
 *   cb_filter_export_bools  BloomFilter::to_proto (bits clone)   src/bloom.rs:54-58
 *   cb_filter_import_bools  BloomFilter::from_proto              src/bloom.rs:61-63
 *   cb_filter_to_bytes      BloomFilter::to_bytes (prost)        src/bloom.rs:66-70
 *   cb_filter_from_bytes    BloomFilter::from_bytes (prost)      src/bloom.rs:74-77
 *   cb_filter_destroy       Drop for BloomFilter (Vec<bool> free)
 *
 * Error behaviour mirrors the reference's panics as codes: inserting into or
 * probing an m == 0 filter returns CB_EZEROM (`h % 0` panics at
 * src/bloom.rs:36); malformed proto bytes return CB_EDECODE (`unwrap()` panics
 * at src/bloom.rs:75). A Rust shim turns both back into panics.
 *
 * Threading: probes are reentrant and read-only on filters (the reference's
 * concurrent `&self` readers under sstables.read(), src/lib.rs:129). Inserts
 * need exclusive access to the target filter (the reference's `&mut self`).
 */
#ifndef CASSBLOOM_H
#define CASSBLOOM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CB_OK 0
#define CB_EINVAL (-1)  /* bad argument (null pointer, bad offsets, ...) */
#define CB_EZEROM (-2)  /* m == 0: the reference panics with `% 0` */
#define CB_ENOMEM (-3)  /* device or host allocation failed */
#define CB_EHIP (-4)    /* HIP runtime error */
#define CB_EDECODE (-5) /* malformed BloomProto bytes */
#define CB_ENODEV (-6)  /* no usable gfx950 device */
#define CB_EUTF8 (-7)   /* a data-file key is not UTF-8: SsTable::load returns Err */

typedef struct cb_filter cb_filter;
typedef struct cb_filterset cb_filterset; /* bit-sliced filter sets, see below */
typedef struct cb_table cb_table;         /* an SSTable data file in HBM, see below */

/* ---- device / library ---- */
int cb_init(int device);
int cb_device_count(int* out);
const char* cb_last_error(void);
const char* cb_version(void);
int cb_stream_synchronize(void* stream);
/* The caller is done with `stream` (call before hipStreamDestroy, with no
 * library call on it in flight): waits for the stream's queued work, frees
 * the per-stream buffers the library keeps for it (keys staging, partition
 * scratch, search outputs) and forgets it. Destroying handles never waits for
 * the device: a filter, table or set's memory is retired behind an event on
 * every stream the library has seen and reused once they have all passed
 * them, so a stream destroyed without this call makes the next destroy fall
 * back to a device-wide synchronise. Ends no work of the caller's. */
int cb_stream_release(void* stream);
/* Pinned (page-locked, device-mapped) host memory for key and hit buffers:
 * FilterSet probes whose keys AND hits live in it run zero-copy (see
 * cb_set_probe_fixed). For callers without the HIP runtime (the Rust shim,
 * INTEGRATION.md §4). */
int cb_host_alloc(uint64_t bytes, void** out);
int cb_host_free(void* p);

/* ---- filter lifetime (BloomFilter::new / Drop) ---- */
/* m_bits may be 0 (legal in the reference; inserts/probes then fail with
 * CB_EZEROM). The filter starts all-zero. */
int cb_filter_create(uint64_t m_bits, int device, cb_filter** out);
int cb_filter_destroy(cb_filter* f);
int cb_filter_bits(const cb_filter* f, uint64_t* m_out);
int cb_filter_device(const cb_filter* f, int* device_out);
/* Device pointer to the packed words (ceil(m/32) uint32 LSB-first, padded
 * with zero words to the allocation). Read-only use by callers. */
int cb_filter_words(const cb_filter* f, const uint32_t** words_out, uint64_t* nwords_out);
int cb_filter_clear(cb_filter* f, void* stream);

/* ---- build (BloomFilter::insert, batched) ---- */
/* n keys of key_len bytes each, contiguous. key_len may be 0. */
int cb_filter_insert_fixed(cb_filter* f, const uint8_t* keys, uint32_t key_len, uint64_t n,
                           void* stream);
/* n ragged keys: key i is bytes[offsets[i] .. offsets[i+1]) (offsets: n+1
 * non-decreasing uint64). */
int cb_filter_insert_var(cb_filter* f, const uint8_t* bytes, const uint64_t* offsets,
                         uint64_t n, void* stream);

/* Concurrent flush builds: filters[i] += keys[i][0 .. n[i]) (key_len bytes
 * each), all filters of one m on one device, built together (one partition
 * and one tile launch per 64 filters). Each keys[i] may be host or device. */
int cb_filter_insert_fixed_many(cb_filter* const* filters, uint32_t nf, const uint8_t* const* keys,
                                uint32_t key_len, const uint64_t* n, void* stream);

/* ---- probe (BloomFilter::may_contain over many filters, batched) ---- */
/* hits: [nf][ceil(n/64)] uint64; bit k%64 of word [f][k/64] is
 * filters[f].may_contain(key k). Tail bits of the last word are zero. Filters
 * may have different m; all must live on the same device. */
int cb_probe_fixed(const cb_filter* const* filters, uint32_t nf, const uint8_t* keys,
                   uint32_t key_len, uint64_t n, uint64_t* hits, void* stream);
int cb_probe_var(const cb_filter* const* filters, uint32_t nf, const uint8_t* bytes,
                 const uint64_t* offsets, uint64_t n, uint64_t* hits, void* stream);
/* Single-key may_contain (host key, synchronous). *out = 0/1. The per-key
 * call of SsTable::get (src/sstable.rs:138) answers from a host mirror of the
 * filter's packed words when the mirror is on: the first call after a write
 * (build, import, clear) waits for that write's stream position and copies
 * ceil(m/32) words back once; later calls are two host word loads, no GPU
 * round trip. With the mirror off every call is a one-key GPU probe.
 * Reentrant: concurrent callers may share a filter (`&self`). */
int cb_may_contain(const cb_filter* f, const uint8_t* key, uint64_t len, int* out);
/* Host mirror policy: 1 on, 0 off, -1 auto (the default: on when m <= 2^24,
 * i.e. up to 2 MiB of host words). With the mirror on every write records an
 * event and the first refresh waits for it. A write made with the mirror off
 * records nothing (it costs the write's stream no event); the first refresh
 * after the mirror is turned on then waits, by events, for the work queued
 * on every stream the library has seen on the device: never for a stored
 * stream handle and never for the whole device, unless such a stream was
 * destroyed without cb_stream_release (then its handle is invalid and the
 * refresh synchronises the device). */
int cb_filter_host_mirror(cb_filter* f, int mode);
/* *on = whether cb_may_contain uses the mirror; *current = whether the mirror
 * already holds the latest write (either may be NULL). Host only. */
int cb_filter_host_mirror_info(const cb_filter* f, int* on, int* current);

/* ---- persistence (to_proto / from_proto / to_bytes / from_bytes) ---- */
/* Vec<bool> layout: m bytes of 0/1. */
int cb_filter_export_bools(const cb_filter* f, uint8_t* out, void* stream);
/* Replaces the filter's contents; m must equal the filter's m. */
int cb_filter_import_bools(cb_filter* f, const uint8_t* in, uint64_t m, void* stream);
/* Packed layout: ceil(m/32) uint32 words (bits >= m in the last word are 0). */
int cb_filter_export_packed(const cb_filter* f, uint32_t* out, void* stream);
int cb_filter_import_packed(cb_filter* f, const uint32_t* in, uint64_t nwords, void* stream);
/* prost encoding of `BloomProto { repeated bool bits = 1; }` (packed): the
 * exact bytes of BloomFilter::to_bytes. Writes at most `cap` bytes; *len_out
 * always receives the full length (call with out=NULL, cap=0 to size). */
int cb_filter_to_bytes(const cb_filter* f, uint8_t* out, uint64_t cap, uint64_t* len_out);
/* BloomFilter::from_bytes: decodes (packed or unpacked elements, unknown
 * fields skipped) into a new filter on `device`. */
int cb_filter_from_bytes(const uint8_t* in, uint64_t len, int device, cb_filter** out);

/* ---- TableMeta: the SSTable `.meta` file ----
 *   message TableMeta { optional BloomProto bloom = 1;          src/sstable.rs:31-37
 *                       optional ZoneMapProto zone_map = 2; }
 *   message ZoneMapProto { optional string min = 1; optional string max = 2; }
 *                                                               src/zonemap.rs:11-17 */
typedef struct cb_zone_bounds {
  const uint8_t* min;
  uint64_t min_len;
  int has_min; /* 0: None */
  const uint8_t* max;
  uint64_t max_len;
  int has_max;
} cb_zone_bounds;
typedef struct cb_meta_info {
  int has_bloom; /* 0: no bloom field; the returned filter is BloomFilter::new(1024) */
  int has_zone;  /* 0: no zone_map field (ZoneMap::default()) */
  cb_zone_bounds zone; /* min/max point INTO the decoded input buffer */
} cb_meta_info;
/* TableMeta{bloom, zone_map}.encode (SsTable::create, src/sstable.rs:74-81).
 * bloom NULL / zone NULL omit that field. The filter's bits are expanded to
 * the prost 0/1 bytes on the device. out may be host or device memory;
 * *len_out is always the encoded length, bytes are written only if cap
 * suffices. CB_EINVAL if a zone bound is not UTF-8. */
int cb_meta_encode(const cb_filter* bloom, const cb_zone_bounds* zone, uint8_t* out, uint64_t cap,
                   uint64_t* len_out);
/* TableMeta::decode + the map()s of SsTable::load (src/sstable.rs:96-108):
 * prost merge semantics (repeated bloom fields append bits, zone strings are
 * last-wins, unknown fields skipped, strings must be UTF-8). CB_EDECODE on a
 * malformed message — the reference then rebuilds from the data file
 * (src/sstable.rs:109-120). The new filter lives on `device`. */
int cb_meta_decode(const uint8_t* in, uint64_t len, int device, cb_filter** bloom_out,
                   cb_meta_info* info);
/* Restart path for a set: decode one table's `.meta` straight into `slot`
 * (filter bits and zone map). The table's m must equal the set's m. */
int cb_set_load_meta(cb_filterset* set, uint32_t slot, const uint8_t* in, uint64_t len,
                     void* stream);

/* ---- bit-sliced filter sets (the read-path fan-out) ---- */
/* A FilterSet holds up to `width` filters of one size m in a position-major
 * layout: word p (uint32 / uint64) has bit s = bit p of the filter in slot s.
 * Probing it answers may_contain for every slot with two word reads per key
 * (Database::get's per-table loop, src/lib.rs:129-134, collapsed; m is
 * uniform across SSTables, src/sstable.rs:44,59). The set is a derived copy:
 * the cb_filter handles stay the source of truth.
 * width is 32, 64, or a multiple of 64 up to 4096 (a "wide" set: row p is
 * width/64 uint64 words, 128 B per row at 1024 slots; at the product's
 * m = 1024 the whole set is 128 KiB). A wide set serves the reference's
 * real shape — a table per 1024 inserts (src/lib.rs:72,105), hundreds of
 * m = 1024 filters — in one launch: cb_set_get_many_* take up to `width`
 * tables. Its probe reads row b's word only where row a's is non-zero (the
 * reference's `&&`, src/bloom.rs:50). cb_set_probe_pack_fixed takes sets of
 * at most 64 slots; cb_set_probe_allgather_fixed takes wide sets when every
 * rank's shard is past 64 rows (below). */
int cb_set_create(uint64_t m_bits, uint32_t width, int device, cb_filterset** out);
int cb_set_destroy(cb_filterset* set);
/* used = 1 + the highest slot assigned so far (the number of hit rows). */
int cb_set_info(const cb_filterset* set, uint64_t* m_out, uint32_t* width_out, uint32_t* used_out);
/* slot := f's bits (f->m must equal the set's m). O(set bits) when the slot is
 * empty (the LSM case: a new SSTable takes a free slot), a full pass otherwise. */
int cb_set_assign(cb_filterset* set, uint32_t slot, const cb_filter* f, void* stream);
/* slots 0..nf-1 := filters[0..nf-1], other slots cleared; used = nf. */
int cb_set_assign_all(cb_filterset* set, const cb_filter* const* filters, uint32_t nf, void* stream);
int cb_set_clear_slot(cb_filterset* set, uint32_t slot, void* stream);
/* hits: [used][ceil(n/64)] uint64, row s = slot s's may_contain bits.
 * Pinned host keys AND hits (hipHostMalloc / torch pin_memory) of fixed-length
 * keys take the zero-copy path: the probe kernel loads the keys and stores the
 * hit rows over PCIe itself (both directions and the HBM gathers overlap in one
 * launch); the call returns when the hits are in host memory. */
int cb_set_probe_fixed(const cb_filterset* set, const uint8_t* keys, uint32_t key_len, uint64_t n,
                       uint64_t* hits, void* stream);
int cb_set_probe_var(const cb_filterset* set, const uint8_t* bytes, const uint64_t* offsets,
                     uint64_t n, uint64_t* hits, void* stream);

/* ---- zone maps and the SsTable::get gate ----
 * Each slot may carry its table's ZoneMap (src/zonemap.rs:3-8: optional
 * min/max key, compared byte-wise like Rust's str Ord). A slot whose zone
 * lacks either bound accepts every key (zonemap.rs:37-42). cb_set_assign,
 * cb_set_assign_all and cb_set_clear_slot reset the slot's zone to "none";
 * set the zone after assigning the table's filter. Zone updates wait for
 * `stream` (they happen once per flush). */
/* The slot's zone := {min, max} — ZoneMap::from_proto (zonemap.rs:55-61). */
int cb_set_zone(cb_filterset* set, uint32_t slot, const uint8_t* min, uint64_t min_len,
                int has_min, const uint8_t* max, uint64_t max_len, int has_max, void* stream);
/* Reads the slot's zone back (to_proto, zonemap.rs:46-52). Bytes are copied
 * only when the buffer is large enough; lengths are always written. */
int cb_set_zone_get(const cb_filterset* set, uint32_t slot, uint8_t* min, uint64_t min_cap,
                    uint64_t* min_len, int* has_min, uint8_t* max, uint64_t max_cap,
                    uint64_t* max_len, int* has_max);
/* ZoneMap::update for every key of a batch, on the device (the zone half of
 * SsTable::create's loop, src/sstable.rs:62-65). n == 0 leaves it as is. */
int cb_set_zone_from_keys_fixed(cb_filterset* set, uint32_t slot, const uint8_t* keys,
                                uint32_t key_len, uint64_t n, void* stream);
int cb_set_zone_from_keys_var(cb_filterset* set, uint32_t slot, const uint8_t* bytes,
                              const uint64_t* offsets, uint64_t n, void* stream);
/* Index of the first lexicographically smallest / largest key of a batch
 * (UINT64_MAX when n == 0). */
int cb_zone_bounds_fixed(const uint8_t* keys, uint32_t key_len, uint64_t n, int device,
                         uint64_t* min_idx, uint64_t* max_idx, void* stream);
int cb_zone_bounds_var(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, int device,
                       uint64_t* min_idx, uint64_t* max_idx, void* stream);
/* SsTable::get's gate for every (key, slot): bit set iff
 * zone_map.contains(key) && bloom.may_contain(key) (src/sstable.rs:138).
 * Same hits layout as cb_set_probe_*. */
int cb_set_probe_gated_fixed(const cb_filterset* set, const uint8_t* keys, uint32_t key_len,
                             uint64_t n, uint64_t* hits, void* stream);
int cb_set_probe_gated_var(const cb_filterset* set, const uint8_t* bytes, const uint64_t* offsets,
                           uint64_t n, uint64_t* hits, void* stream);

/* ---- SSTable data files and the batched read path ----
 * A data file is SsTable::create's output (src/sstable.rs:57-72): lines
 * `key \t base64(value) \n` sorted by key. cb_table_create uploads one (host
 * or device bytes) and indexes its lines on the device exactly as SsTable::get
 * splits them (raw.split('\n') minus empty lines, src/sstable.rs:142-146). */
int cb_table_create(const uint8_t* data, uint64_t len, int device, void* stream, cb_table** out);
int cb_table_destroy(cb_table* t);
/* Device pointer to the file bytes (valid until cb_table_destroy) and length. */
int cb_table_data(const cb_table* t, const uint8_t** data, uint64_t* len);
/* Copies file bytes [offset, offset+len) to out (host or device), synchronous:
 * what storage.put(&path, data) writes (src/sstable.rs:73). */
int cb_table_copy(const cb_table* t, uint64_t offset, uint64_t len, uint8_t* out);
/* SsTable::create (src/sstable.rs:51-87) on the device, for n entries given as
 * ragged key and value arrays (host or device): stable sort by key (skipped
 * when already sorted, as memtable flushes are), the data file `key \t
 * STANDARD.encode(value) \n` (*table_out, indexed and searchable), the
 * table's Bloom filter of m_bits (*bloom_out, nullable: BloomFilter::new(1024)
 * + insert per key in the reference) and its zone map as the input indices of
 * a smallest and a largest key (UINT64_MAX when n == 0).
 * The call only ENQUEUES its work on `stream` (the device decides whether the
 * batch needs a sort) and returns; the table finalises on first use — every
 * call that reads it (cb_table_*, searches, get_many, cb_table_wait) first
 * waits for the work and takes its results once. zone_min_idx / zone_max_idx
 * non-NULL are host results: the call then waits itself. Device offsets cost
 * one read-back of their totals (cb_sstable_create_bounded takes bounds
 * instead). Host inputs are staged into memory the table owns; device inputs
 * must stay valid until the table is finalised (a batch the bin sort cannot
 * place — keys sharing long prefixes — is sorted again from them then). */
int cb_sstable_create(const uint8_t* keys, const uint64_t* key_off, const uint8_t* vals,
                      const uint64_t* val_off, uint64_t n, uint64_t m_bits, int device, void* stream,
                      cb_table** table_out, cb_filter** bloom_out, uint64_t* zone_min_idx,
                      uint64_t* zone_max_idx);
/* The same, enqueue-only for device offsets too: key_bytes / val_bytes bound
 * key_off[n] / val_off[n] (the file buffer is sized from them). A batch past
 * its bounds writes no file; its table reports CB_EINVAL when finalised, and
 * the Bloom filter returned with it must be discarded (device offsets past a
 * device buffer's end are the caller's error, as for any device pointer).
 * Host key or value bytes with device offsets are checked before the call
 * returns (one read-back of the offsets' totals): the bytes are staged into a
 * block of exactly key_bytes / val_bytes, so a batch past them is refused
 * with CB_EINVAL and nothing is enqueued. */
int cb_sstable_create_bounded(const uint8_t* keys, const uint64_t* key_off, uint64_t key_bytes, const uint8_t* vals,
                              const uint64_t* val_off, uint64_t val_bytes, uint64_t n, uint64_t m_bits, int device,
                              void* stream, cb_table** table_out, cb_filter** bloom_out);
/* Finalise a table from cb_sstable_create*: wait for its work, take its
 * results; returns its deferred error, if any. Idempotent, thread-safe. */
int cb_table_wait(const cb_table* t);
/* The zone map bounds of a table made by cb_sstable_create with n >= 1 (the
 * first / last key of the file: ZoneMap::update over the sorted entries,
 * src/sstable.rs:60-64): which = 0 min, 1 max. *len = the key's length; up to
 * cap bytes are copied to host memory out. Host only, no device access.
 * CB_EINVAL for other tables. */
int cb_table_zone(const cb_table* t, int which, uint8_t* out, uint64_t cap, uint64_t* len);
int cb_table_info(const cb_table* t, uint64_t* nlines, uint64_t* bytes);
/* SsTable::load's rebuild when the `.meta` file is missing or undecodable
 * (src/sstable.rs:109-120), on the device from the table's line index: a new
 * filter of m_bits (BloomFilter::new(1024) in the reference) holding the key
 * of every line that has a TAB (bytes before the first TAB; lines without one
 * are skipped), and the zone map over the same keys, returned as the line
 * indices of a smallest and a largest key (UINT64_MAX when no line has a
 * TAB; cb_table_lines + cb_table_copy give the bytes). CB_EUTF8 when a key is
 * not UTF-8 (the reference's load returns Err; nothing is returned then). */
int cb_table_rebuild(const cb_table* t, uint64_t m_bits, void* stream, cb_filter** bloom_out,
                     uint64_t* zone_min_line, uint64_t* zone_max_line);
/* *out = 1 when the file is well-formed (a TAB on every line, keys strictly
 * increasing — what SsTable::create writes): then any correct search gives
 * the reference's answer and the prefix/fence index is used; otherwise the
 * exact (lo+hi)/2 trajectory of src/sstable.rs:163-177 is replayed. */
int cb_table_well_formed(const cb_table* t, int* out);
/* Tests/bench: tables created while on != 0 always use the exact trajectory. */
int cb_table_force_exact(int on);
/* The read path's key buckets (136 B per line, rounded up to a power of two
 * lines: 64 MiB for 512K lines, 2.3 GiB for 2^24) are built for a table only
 * when they take at most max_bytes AND at most a quarter of the device memory
 * free when they are built; otherwise that table is searched without them
 * (same answers, ~20 % slower reads). max_bytes = 0 turns them off for tables
 * read from now on; the default is 1 GiB. Process-wide. */
int cb_table_bucket_limit(uint64_t max_bytes);
/* The line index: start offset, key length (bytes before the first TAB, or
 * UINT32_MAX when the line has none) and line length; host or device out. */
int cb_table_lines(const cb_table* t, uint64_t* start, uint32_t* key_len, uint32_t* line_len);
/* SsTable::binary_search (src/sstable.rs:161-179) for a key batch, same
 * (lo+hi)/2 trajectory: line_out[k] = matching line index or -1. */
int cb_table_search_fixed(const cb_table* t, const uint8_t* keys, uint32_t key_len, uint64_t n,
                          int64_t* line_out, void* stream);
int cb_table_search_var(const cb_table* t, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                        int64_t* line_out, void* stream);
/* Database::get's table walk (src/lib.rs:128-134) for a key batch.
 * tables[0] is the NEWEST table. hits (nullable): the per-table gate from a
 * (gated) probe, [rows][ceil(n/64)] with table t in row hit_rows[t] (hit_rows
 * NULL = row t); a table is searched for key k only where its bit is set.
 * which[k] = index of the first table whose SsTable::get returns Ok(Some) —
 * line found AND value decodes as base64 (base64 0.21.7 STANDARD; an Err
 * falls through to older tables) — or -1. val_off[n+1] = offsets of the
 * decoded values; *total = their byte count; the values are written to vals
 * only if cap >= *total (call with vals = NULL to size).
 * total = NULL: the call only enqueues the work on stream and returns without
 * waiting (keys, hits, which, val_off and vals must then be device memory;
 * val_off[n] holds the total once the stream has run, and vals is written
 * only if cap >= that total). Calls that repeat the same tables and hit_rows
 * upload nothing, so batches on two streams overlap. A well-formed table's
 * first get_many (this or cb_set_get_many) also enqueues the build of its key
 * buckets on that call's stream (device memory: 136 B per line, rounded up
 * to a power of two lines; freed with the table) when they fit the budget
 * set by cb_table_bucket_limit; later calls on any stream enqueue a wait for
 * that build (never a host wait) until it is seen complete. */
int cb_get_many_fixed(const cb_table* const* tables, uint32_t nt, const uint64_t* hits,
                      const uint32_t* hit_rows, const uint8_t* keys, uint32_t key_len, uint64_t n,
                      int32_t* which, uint64_t* val_off, uint8_t* vals, uint64_t cap,
                      uint64_t* total, void* stream);
int cb_get_many_var(const cb_table* const* tables, uint32_t nt, const uint64_t* hits,
                    const uint32_t* hit_rows, const uint8_t* bytes, const uint64_t* offsets,
                    uint64_t n, int32_t* which, uint64_t* val_off, uint8_t* vals, uint64_t cap,
                    uint64_t* total, void* stream);
/* Database::get in one launch (src/lib.rs:125-136 with SsTable::get's gate,
 * src/sstable.rs:138): the same walk and outputs as cb_get_many_*, with each
 * (key, table) gate — zone_map.contains && bloom.may_contain, exactly
 * cb_set_probe_gated_*'s bit — computed from the FilterSet inside the search
 * kernel instead of read from hit rows. Table t is set slot slots[t]
 * (slots NULL = slot t); nt <= the set's width (up to 4096 with a wide set;
 * runs of ascending or descending slots, e.g. slot = the table's position in
 * Vec<SsTable> walked newest first, take each group of 64 tables' gate from
 * one window of the set's rows, other mappings one bit per table); tables and
 * set on one device. Same async contract (total = NULL). */
int cb_set_get_many_fixed(const cb_filterset* set, const cb_table* const* tables, uint32_t nt,
                          const uint32_t* slots, const uint8_t* keys, uint32_t key_len, uint64_t n,
                          int32_t* which, uint64_t* val_off, uint8_t* vals, uint64_t cap, uint64_t* total,
                          void* stream);
int cb_set_get_many_var(const cb_filterset* set, const cb_table* const* tables, uint32_t nt,
                        const uint32_t* slots, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                        int32_t* which, uint64_t* val_off, uint8_t* vals, uint64_t cap, uint64_t* total,
                        void* stream);

/* ---- multi-GPU exchange ----
 * Each rank holds hit rows [rows][words] (uint64) for its filter subset; the
 * ranks all-gather them so every rank has the [total_rows][words] map that
 * Database::get's fan-out reads (src/lib.rs:129-134). At BASELINE densities
 * the rows are sparse, so a rank can ship the positions of its set bits:
 *   cb_hits_pack_words: size in uint32 of a pack for rows x words of hits and
 *     cap positions: 2 + cap + 2 * ceil(rows * words / 2048). Packs that are
 *     all-gathered must all have the size of the LARGEST shard's pack.
 *   cb_hits_compress: pack := {count, 0, positions[cap], directory}; position
 *     = row * words * 64 + bit; the rows are cut into blocks of 2048 words and
 *     directory entry b = {first slot, number} of block b's positions
 *     (ascending inside the block). One launch. count may exceed cap: the
 *     pack is then incomplete (which positions were kept is unspecified) and
 *     all ranks must fall back to the dense exchange.
 *     Requires rows * words * 64 < 2^32. Device pointers, async on stream.
 *   cb_hits_expand: full := the dense map holding the positions of packs[r]
 *     (nranks packs, all-gathered with the stride cb_hits_pack_words gives for
 *     the largest shard) at global row row_off[r] (host array, row_off[0] = 0,
 *     non-decreasing, nranks <= 64; rank r has rows up to row_off[r+1], the
 *     last up to total_rows); every word of full is written once. Bit-identical
 *     to the dense all-gather when no rank's count exceeds cap. A rank whose
 *     count exceeds cap contributes zeros and clears *ok (a device uint32, may
 *     be NULL): the overflow report is asynchronous, so the caller checks ok
 *     before using full and redoes that batch's exchange densely when it is 0. */
int cb_hits_pack_words(uint64_t rows, uint64_t words, uint64_t cap, uint64_t* out);
int cb_hits_compress(const uint64_t* hits, uint64_t rows, uint64_t words, uint32_t* pack,
                     uint64_t cap, void* stream);
int cb_hits_expand(const uint32_t* packs, uint32_t nranks, uint64_t cap, const uint64_t* row_off,
                   uint64_t words, uint64_t total_rows, uint64_t* full, uint32_t* ok, void* stream);

/* The whole exchange behind one call, over RCCL (one process per GPU, xGMI
 * between the GPUs of a node). Replaces the per-table loop of Database::get
 * (src/lib.rs:129-134) when the tables' filters are sharded over GPUs: the
 * table subset of rank r is rows [first_row, first_row + rows) of the global
 * map, as cb_comm_shard splits total_rows (contiguous, sizes differ by <= 1,
 * larger shards first).
 *   cb_comm_unique_id: rank 0 makes the 128-byte id and hands it to every
 *     rank by any channel (the Rust store: its own RPC; Python: the process
 *     group's broadcast).
 *   cb_comm_init: collective over the `world` ranks; binds to `device`. The
 *     calling thread's current device is left unchanged.
 *   cb_hits_allgather: collective. local = this rank's [rows][words] uint64
 *     hits (rows = its shard of total_rows), full = the [total_rows][words]
 *     map, both device memory on the communicator's device; async on stream.
 *     mode CB_XCHG_DENSE: one all-gather of the rows. CB_XCHG_SPARSE: compress
 *     -> all-gather of (2 + cap)-word packs -> expand (cap > 0, the same on
 *     every rank). With ok == NULL the gathered counts are read back (the
 *     stream is synchronised) and, if any rank's set bits exceed cap, every
 *     rank redoes the batch densely: full is always complete. With ok != NULL
 *     (a device uint32 holding 1) nothing is read back: ok is cleared when a
 *     rank overflowed, and the caller redoes that batch with CB_XCHG_DENSE.
 *     *sparse_used (nullable) = 1 when the map came from the packs.
 *   Exchanges on one communicator must be issued in the same order on every
 *   rank. They may come from several streams (pipelined batches): the
 *   library keeps a buffer set per stream and runs a communicator's
 *   collectives one after another in issue order (each waits for an event
 *   recorded after the previous one), so at most one collective of a
 *   communicator is in flight and no two communicators' collectives need to
 *   interleave. Use ONE communicator per rank. */
#define CB_COMM_ID_BYTES 128
#define CB_XCHG_DENSE 0
#define CB_XCHG_SPARSE 1
typedef struct cb_comm cb_comm;
int cb_comm_unique_id(uint8_t* id /* CB_COMM_ID_BYTES */);
int cb_comm_init(int rank, int world, const uint8_t* id, int device, cb_comm** out);
/* Two more transports under the same collectives (every host and device step
 * of cb_hits_allgather / cb_set_probe_allgather_fixed is shared; only the
 * all-gather of bytes differs):
 *   cb_comm_init_loopback: `world` ranks in ONE process on one device;
 *     ranks[r] (an array of world handles) is rank r's communicator. Each
 *     rank's collectives must be issued from its own host thread: a call
 *     returns once every rank has issued it. The all-gather is device copies
 *     between the ranks' buffers, ordered by events on each caller's stream.
 *     For tests of world > 1 on one GPU.
 *   cb_comm_init_host: the caller moves the bytes (its own RPC, MPI, gloo ...):
 *     the library synchronises the stream, copies this rank's `bytes` of send
 *     data to host memory, calls fn(user, send, recv, bytes) — fn must leave
 *     rank r's bytes at recv + r * bytes for every rank and return 0 — and
 *     copies recv back to the device. Not collective at init. */
typedef int (*cb_host_allgather_fn)(void* user, const void* send, void* recv, uint64_t bytes);
int cb_comm_init_loopback(int world, int device, cb_comm** ranks);
int cb_comm_init_host(int rank, int world, int device, cb_host_allgather_fn fn, void* user,
                      cb_comm** out);
int cb_comm_destroy(cb_comm* c);
/* Ends the communicator on this rank (ncclCommAbort for RCCL; a loopback
 * group wakes every rank): callable from any thread, also while another
 * thread is blocked inside a collective of c, which then returns an error.
 * Every later exchange on c fails with CB_EINVAL; cb_comm_destroy still
 * frees the handle. For a rank's watchdog: a peer that never joins a
 * collective would otherwise hold this rank forever. */
int cb_comm_abort(cb_comm* c);
int cb_comm_info(const cb_comm* c, int* rank, int* world, int* device);
int cb_comm_shard(uint64_t total_rows, int world, int rank, uint64_t* first_row, uint64_t* rows);
int cb_hits_allgather(cb_comm* c, const uint64_t* local, uint64_t rows, uint64_t words,
                      uint64_t total_rows, uint64_t* full, int mode, uint64_t cap, uint32_t* ok,
                      int* sparse_used, void* stream);

/* The probe and the exchange in one call: this rank's FilterSet probe (its
 * `used` slots must equal its shard of total_rows) of a device-resident batch
 * of fixed-length keys, writing local_hits ([used][ceil(n/64)], device), then
 * the all-gather into full. In sparse mode the probe kernel itself writes the
 * pack (no separate compress pass): positions as cb_hits_compress's, with
 * one directory entry per probe block of 16 hit words of every slot
 * (cb_set_pack_words). ok / sparse_used / overflow as cb_hits_allgather.
 * gated != 0 applies the zone gate (cb_set_probe_gated_fixed). When the
 * largest shard passes 64 rows (wide sets), sparse mode probes first and
 * then runs cb_hits_allgather's sparse exchange (a separate compress pass);
 * every rank must then hold such a shard, as the shard split guarantees. */
int cb_set_probe_allgather_fixed(cb_comm* c, const cb_filterset* set, const uint8_t* keys, uint32_t key_len,
                                 uint64_t n, int gated, uint64_t* local_hits, uint64_t total_rows,
                                 uint64_t* full, int mode, uint64_t cap, uint32_t* ok, int* sparse_used,
                                 void* stream);
/* Its pieces, for callers that move the packs themselves: the pack size for
 * a batch of n keys and cap positions (2 + cap + 2 * ceil(ceil(n/64)/16)
 * uint32); the probe writing hits and pack (device buffers, async); and the
 * expand of nranks such packs (all-gathered, each of cb_set_pack_words) into
 * the [total_rows][ceil(n/64)] map, rank r's rows starting at row_off[r]
 * (<= 64 rows per rank). A rank whose count exceeds cap clears *ok and
 * leaves its rows zero. */
int cb_set_pack_words(uint64_t n, uint64_t cap, uint64_t* out);
int cb_set_probe_pack_fixed(const cb_filterset* set, const uint8_t* keys, uint32_t key_len, uint64_t n, int gated,
                            uint64_t* hits, uint32_t* pack, uint64_t cap, void* stream);
int cb_hits_expand_set(const uint32_t* packs, uint32_t nranks, uint64_t cap, const uint64_t* row_off, uint64_t n,
                       uint64_t total_rows, uint64_t* full, uint32_t* ok, void* stream);

/* ---- tuning / introspection (bench + tests) ---- */
/* Path selection: 0 = auto, 1 = force direct (per-key atomics / gathers),
 * 2 = force tiled (LDS-staged filter tiles). Process-wide. */
int cb_set_path(int path);
/* FilterSet probes of dense batches (at least 2 keys per 128-B line of the
 * set: the C5 shape) take the region-partitioned probe, which streams the set
 * through LDS once instead of reading a random line per key; same hits.
 * mode 0 = by density (default), 1 = whenever the set allows it (32- or
 * 64-slot sets, m <= 2^32 in at most 4096 regions of 64 KiB; tests), -1 =
 * never. Never for gated probes or the fused exchange pack. Process-wide. */
int cb_set_dense(int mode);
/* Path the last insert/probe on this thread used (1 direct, 2 tiled, 3 FilterSet,
 * 4 FilterSet zero-copy: pinned host keys and hits read/written by the kernel,
 * 5 cb_may_contain answered from the host mirror, 6 FilterSet dense probe). */
int cb_last_path(void);
/* Per-kernel timing with HIP events recorded on each launch's own stream
 * (off by default). Kernel names: "k_insert_direct", "k_probe_direct",
 * "k_build_part", "k_build_tile", "k_part_probe", "k_tile_probe",
 * "k_masks_to_hits", "k_set_build", "k_set_or_slot", "k_set_put_slot",
 * "k_set_probe". cb_profile_read waits for pending events and returns the
 * accumulated milliseconds and launch count for one kernel. */
int cb_profile_enable(int on);
int cb_profile_reset(void);
int cb_profile_read(const char* kernel, double* total_ms, uint64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* CASSBLOOM_H */
