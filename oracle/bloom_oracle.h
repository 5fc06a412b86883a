/*
 * bloom_oracle.h — CPU restatement of the reference Bloom filter.
 *
 * TEST INFRASTRUCTURE ONLY. This is the parity checker for the HIP path in
 * lsmt_amd/csrc. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it. The product path (libcassbloom.so) never
 * links, calls or falls back to it.
 *
 * Restates /root/reference/src/bloom.rs (mweiden/lsmt, crate `cass`):
 *   storage    : one byte per bit, 0/1         (Vec<bool>, src/bloom.rs:4-7,17-21)
 *   hashes     : u64 wrapping djb2 (x33, seed 5381) and x31 (seed 0) over
 *                the key's bytes, index = h % m  (src/bloom.rs:26-37)
 *   insert     : sets bits[a] and bits[b]       (src/bloom.rs:40-44)
 *   may_contain: bits[a] && bits[b], short-circuit (src/bloom.rs:48-51)
 *   to/from_bytes: prost encoding of `repeated bool bits = 1` (packed)
 *                  (src/bloom.rs:9-13,54-77)
 *
 * Parity pinning: the Rust reference cannot be compiled in this image (no
 * cargo/rustc). This restatement is pinned by the reference's own test
 * assertions (tests/bloom_test.rs:3-8, tests/sstable_local_test.rs:12) and by
 * known-answer vectors from an independent Python big-int restatement
 * (tests/golden/make_golden.py). See DESIGN.md "Parity".
 */
#ifndef CASSBLOOM_ORACLE_H
#define CASSBLOOM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OB_OK 0
#define OB_EINVAL (-1)
#define OB_EZEROM (-2)   /* reference panics: `h % 0` at src/bloom.rs:36 */
#define OB_ENOMEM (-3)
#define OB_EDECODE (-5)  /* reference panics: `decode(..).unwrap()` at src/bloom.rs:75 */
#define OB_EUTF8 (-7)    /* SsTable::load returns Err: a data-file key is not UTF-8 */

typedef struct ob_filter {
  uint8_t* bits; /* m bytes, each 0 or 1 — the Vec<bool> layout */
  uint64_t m;
} ob_filter;

/* BloomFilter::new(size) — src/bloom.rs:17-21. m == 0 is legal (the panic is
 * deferred to the first hashes() call, as in the reference). */
int ob_new(ob_filter* f, uint64_t m);
void ob_free(ob_filter* f);

/* The two raw u64 hashes before the modulo — src/bloom.rs:28-34. */
void ob_raw_hashes(const uint8_t* key, uint64_t len, uint64_t* h1, uint64_t* h2);
/* hashes(): (h1 % m, h2 % m) — src/bloom.rs:35-36. OB_EZEROM if m == 0. */
int ob_hashes(const uint8_t* key, uint64_t len, uint64_t m, uint64_t* a, uint64_t* b);

int ob_insert(ob_filter* f, const uint8_t* key, uint64_t len);
/* returns 1/0, or OB_EZEROM */
int ob_may_contain(const ob_filter* f, const uint8_t* key, uint64_t len);

/* Batched restatements of the callers' per-key loops:
 * build  — SsTable::create's loop (src/sstable.rs:62-65), keys in order;
 * probe  — Database::get's per-table probe (src/lib.rs:129-134) for every
 *          (key, table) pair. hits is [nf][ceil(n/64)] u64, bit k%64 of word
 *          k/64 set iff filter f may_contain key k; tail bits are zero. */
int ob_insert_fixed(ob_filter* f, const uint8_t* keys, uint32_t key_len, uint64_t n);
int ob_insert_var(ob_filter* f, const uint8_t* bytes, const uint64_t* offsets, uint64_t n);
int ob_probe_fixed(const ob_filter* const* fs, uint32_t nf, const uint8_t* keys,
                   uint32_t key_len, uint64_t n, uint64_t* hits, int threads);
int ob_probe_var(const ob_filter* const* fs, uint32_t nf, const uint8_t* bytes,
                 const uint64_t* offsets, uint64_t n, uint64_t* hits, int threads);

/* prost encoding of BloomProto{bits} (to_bytes, src/bloom.rs:66-70):
 * m == 0 -> empty; else 0x0A, varint(m), m bytes of 0/1. Returns the encoded
 * length; writes only if cap is large enough. */
uint64_t ob_encode(const ob_filter* f, uint8_t* out, uint64_t cap);
/* prost decoding (from_bytes, src/bloom.rs:74-77): accepts packed and
 * unpacked field-1 elements, skips unknown fields; OB_EDECODE on malformed. */
int ob_decode(const uint8_t* in, uint64_t len, ob_filter* out);

/* ZoneMap (/root/reference/src/zonemap.rs:3-42): min/max key seen, compared
 * as Rust compares &str — byte-wise lexicographic, a proper prefix is smaller.
 * contains() is true when either bound is missing (zonemap.rs:37-42). */
typedef struct ob_zone {
  uint8_t* min;
  uint64_t min_len;
  int has_min;
  uint8_t* max;
  uint64_t max_len;
  int has_max;
} ob_zone;
void ob_zone_init(ob_zone* z);
void ob_zone_free(ob_zone* z);
int ob_zone_set(ob_zone* z, const uint8_t* min, uint64_t min_len, int has_min, const uint8_t* max,
                uint64_t max_len, int has_max);
int ob_zone_update(ob_zone* z, const uint8_t* key, uint64_t len);   /* zonemap.rs:21-32 */
int ob_zone_contains(const ob_zone* z, const uint8_t* key, uint64_t len); /* zonemap.rs:37-42 */
int ob_bytes_cmp(const uint8_t* a, uint64_t alen, const uint8_t* b, uint64_t blen);
/* SsTable::get's gate (src/sstable.rs:138) for every (key, table):
 * zone_map.contains(key) && bloom.may_contain(key); zones may be NULL
 * entries (no zone map = accept). Same hits layout as ob_probe_*. */
int ob_probe_gated_var(const ob_filter* const* fs, const ob_zone* const* zones, uint32_t nf,
                       const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint64_t* hits);

/* TableMeta { optional BloomProto bloom = 1; optional ZoneMapProto zone_map = 2; }
 * (src/sstable.rs:31-37), the `.meta` file of an SSTable, and ZoneMapProto
 * { optional string min = 1; optional string max = 2; } (zonemap.rs:11-17).
 * encode (src/sstable.rs:74-81): prost writes a present optional field even
 * when empty; bloom/zone NULL = field absent, a zone bound with has_* = 0 is
 * absent. Returns the encoded length; writes only if cap is large enough.
 * decode (src/sstable.rs:96-108): prost merge semantics — fields in any
 * order, a repeated singular message field merges (BloomProto bits append,
 * ZoneMapProto strings: last wins), unknown fields skipped, strings must be
 * UTF-8. OB_EDECODE on anything malformed (the reference then rebuilds the
 * table's metadata from the data file, src/sstable.rs:109-120). */
typedef struct ob_meta {
  int has_bloom; /* 0: load() uses BloomFilter::new(1024) */
  ob_filter bloom;
  int has_zone; /* 0: load() uses ZoneMap::default() */
  ob_zone zone;
} ob_meta;
uint64_t ob_meta_encode(const ob_filter* bloom, const ob_zone* zone, uint8_t* out, uint64_t cap);
int ob_meta_decode(const uint8_t* in, uint64_t len, ob_meta* out);
void ob_meta_free(ob_meta* m);
int ob_utf8_valid(const uint8_t* p, uint64_t n); /* Rust str::from_utf8 acceptance */

/* SSTable data file (SsTable::create, src/sstable.rs:57-72): sorted lines
 * `key \t base64(value) \n`. ob_table_index restates SsTable::get's
 * raw.split(NL).filter(non-empty) (src/sstable.rs:142-146): line i is
 * data[start[i] .. end[i]). */
typedef struct ob_table {
  const uint8_t* data; /* not owned */
  uint64_t len, nlines;
  uint64_t* start;
  uint64_t* end;
} ob_table;
int ob_table_index(const uint8_t* data, uint64_t len, ob_table* t);
void ob_table_free(ob_table* t);
/* SsTable::binary_search (src/sstable.rs:161-179), same (lo+hi)/2 trajectory:
 * the matching line's index, or -1 (also when the probed line has no TAB,
 * which ends the search). *val / *val_len: the bytes after the TAB. */
int64_t ob_table_search(const ob_table* t, const uint8_t* key, uint64_t klen, uint64_t* val,
                        uint64_t* val_len);
/* SsTable::load's rebuild when the `.meta` file is missing or undecodable
 * (src/sstable.rs:109-120): a fresh BloomFilter of m bits and ZoneMap; for
 * every non-empty line in file order that has a TAB, key = the bytes before
 * the first TAB; a key that is not UTF-8 ends the load with an error
 * (OB_EUTF8, *bad_line = that line); otherwise bloom.insert(key) and
 * zone_map.update(key). Lines without a TAB are skipped. bloom and zone are
 * initialised here; free them with ob_free / ob_zone_free. */
int ob_table_rebuild(const ob_table* t, uint64_t m, ob_filter* bloom, ob_zone* zone, uint64_t* bad_line);
/* base64 0.21.7 STANDARD engine (the reference's `STANDARD.decode`,
 * src/sstable.rs:148): alphabet A-Z a-z 0-9 + /, canonical '=' padding
 * required (length % 4 == 0), non-zero trailing bits rejected. Returns the
 * decoded length, or -1 on any decode error; out may be NULL. */
int64_t ob_b64_decode(const uint8_t* in, uint64_t len, uint8_t* out);
/* STANDARD.encode (src/sstable.rs:69): returns the encoded length. */
uint64_t ob_b64_encode(const uint8_t* in, uint64_t len, uint8_t* out);
/* Database::get's table walk (src/lib.rs:128-134) for a key batch: tables[0]
 * is the NEWEST; hits (nullable, [nt][ceil(n/64)]) is each table's gate
 * (zone && bloom, src/sstable.rs:138). which[k] = first table whose get
 * returns Ok(Some) (found and base64-decodable; a decode Err falls through
 * to older tables), or -1. val_off[n+1] = prefix offsets of the decoded
 * values in vals; vals written only if cap >= *total. */
int ob_get_many(const ob_table* const* tables, uint32_t nt, const uint64_t* hits,
                const uint8_t* bytes, const uint64_t* offsets, uint64_t n, int32_t* which,
                uint64_t* val_off, uint8_t* vals, uint64_t cap, uint64_t* total);

/* SsTable::create's data file (src/sstable.rs:56-72): entries stably sorted
 * by key (sort_by on &str), each written as key \t STANDARD.encode(value) \n.
 * Keys/values are ragged arrays (offsets n+1). Returns the file length;
 * writes only if cap is large enough. */
uint64_t ob_sstable_create(const uint8_t* kbytes, const uint64_t* koff, const uint8_t* vbytes,
                           const uint64_t* voff, uint64_t n, uint8_t* out, uint64_t cap);

/* Synthetic workload keys: 16 lowercase hex chars, MSB
 * nibble first, of splitmix64(seed * 2^32 + i). out is n*16 bytes. */
void ob_gen_keys(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out);
uint64_t ob_splitmix64(uint64_t x);

#ifdef __cplusplus
}
#endif
#endif
