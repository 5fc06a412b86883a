// sstable.hpp — SSTable data files resident in HBM and the batched read-path
// resolution after the Bloom/zone gate.
//
// A data file is SsTable::create's output (/root/reference/src/sstable.rs:
// 57-72): lines `key \t base64(value) \n` sorted by key. SsTable::get
// (src/sstable.rs:133-153) splits it on '\n', drops empty lines, binary-
// searches the lines (161-179) and base64-decodes the hit (148). Database::get
// (src/lib.rs:128-134) asks the tables newest-first and keeps the first
// Ok(Some). Here one lane resolves one key across all its candidate tables.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hash.hpp"
#include "zone.hpp"

namespace cb {

constexpr uint32_t kNoSep = 0xFFFFFFFFu;  // line without a TAB: ends a search

// The prefix index of a well-formed table is a fan-out-16 tree kept as
// levels of sampled prefixes: level 0 is pfx itself, level j >= 1 holds
// pfx[l] for every l that is a multiple of 16^j, up to the first level of at
// most 16 entries. A lookup reads one run of at most 16 consecutive entries
// (one 128-B line) per level. Levels 1..L are stored one after another in
// the fence array.
constexpr uint32_t kFanBits = 4;
constexpr uint32_t kFanout = 1u << kFanBits;
__host__ __device__ inline uint64_t level_count(uint64_t nl, uint32_t j) {
  return (nl + (1ull << (kFanBits * j)) - 1) >> (kFanBits * j);
}
// L: the top level (0 when the table has at most 16 lines)
__host__ __device__ inline uint32_t fence_levels(uint64_t nl) {
  uint32_t L = 0;
  while (level_count(nl, L) > kFanout) ++L;
  return L;
}
// offset of level j >= 1 in the fence array
__host__ __device__ inline uint64_t level_offset(uint64_t nl, uint32_t j) {
  uint64_t o = 0;
  for (uint32_t i = 1; i < j; ++i) o += level_count(nl, i);
  return o;
}
__host__ __device__ inline uint64_t fence_words(uint64_t nl) { return level_offset(nl, fence_levels(nl) + 1); }
// level j >= 1 entry of line l (a multiple of 16^j): fence[level_offset(nl, j) + (l >> 4j)]
__device__ __forceinline__ void fence_put(uint64_t* fence, uint64_t nl, uint64_t l, uint64_t v) {
  const uint32_t L = fence_levels(nl);
  uint64_t off = 0;
  for (uint32_t j = 1; j <= L; ++j) {
    if (l & ((1ull << (kFanBits * j)) - 1)) break;
    fence[off + (l >> (kFanBits * j))] = v;
    off += level_count(nl, j);
  }
}
// Radix directory of a well-formed table: below the prefix bits every line
// shares (dshift = clz(pfx[0] ^ pfx[nlines-1])), the next dbits bits of a
// prefix name its bucket; dir[B] = the first line whose bucket is >= B
// (dir[2^dbits] = nlines). A lookup reads dir[B], dir[B+1]: a bucket of at
// most 8 lines (~4 on average) is searched with one round of prefix loads
// (and its record loaded with them when it holds one line); a larger one
// starts the fence descent at the lowest level where it spans at most 16
// entries. Tables of fewer than 16 lines have none.
constexpr uint32_t kDirLineBits = 2;
__host__ __device__ inline uint32_t dir_bits(uint64_t nl) {
  if (nl < (1ull << (kDirLineBits + 2)) || nl >= (1ull << 32)) return 0;
  const uint32_t b = 63u - (uint32_t)__builtin_clzll(nl) - kDirLineBits;
  return b > 24 ? 24 : b;
}
inline uint64_t dir_words(uint64_t nl) {  // uint32 words
  const uint32_t b = dir_bits(nl);
  return b ? (1ull << b) + 1 : 0;
}
constexpr uint32_t kBadValue = 0xFFFFFFFFu;  // value that STANDARD.decode rejects

// Per-line index record (32 B, one load). vdl is computed once at index
// time: the decoded length of the line's value, or kBadValue when base64
// 0.21.7 STANDARD.decode would fail (or the line has no TAB) — so the read
// path never re-validates a value. pfx2 lets keys of <= 16 bytes be
// compared from the index alone.
struct alignas(16) LineRec {
  uint64_t start;  // line start offset in the file
  uint64_t pfx2;   // key bytes 8..15, big-endian, zero-padded
  uint32_t klen;   // bytes before the first TAB, or kNoSep
  uint32_t llen;   // line length (without the '\n')
  uint32_t vdl;    // decoded value length, or kBadValue
  uint32_t pad;
};

// One data file and its line index. When the file is well-formed — every
// line has a TAB and the keys are strictly increasing, as SsTable::create
// writes it — any correct search returns what the reference's binary search
// returns, so `fast` files are searched through pfx (each key's first 8
// bytes, big-endian, zero-padded: monotone in the key order) and the fence
// levels above it (fence_levels), so a lookup reads one run of at most 16
// entries per level, then the record. Other files replay the exact
// (lo+hi)/2 trajectory.
struct TableView {
  const uint8_t* data;    // the file, with 16 bytes of readable slack
  const LineRec* rec;     // nlines
  const uint64_t* pfx;    // nlines
  const uint64_t* fence;  // fence_words(nlines): levels 1..nlev
  uint64_t nlines;
  uint32_t nlev;          // fence_levels(nlines)
  uint32_t fast;
  const uint32_t* dir;    // dir_words(nlines) (nullptr: none)
  uint32_t dbits;         // dir_bits(nlines)
  uint32_t dshift;        // prefix bits every line shares (64: directory unused)
  uint64_t dp0;           // pfx[0]
};

// ---- line index build: count -> scan -> emit -> finish ----
constexpr uint32_t kLineChunk = 4096;  // bytes per block (256 threads x 16 B)
inline uint64_t line_blocks(uint64_t len) { return (len + kLineChunk - 1) / kLineChunk; }
// cnt[b] = non-empty line starts in chunk b
hipError_t launch_line_count(const uint8_t* data, uint64_t len, uint64_t* cnt, hipStream_t s);
// start[base[b] + j] = j-th line start of chunk b; end[l] = its '\n' (ends of
// the last line at EOF stay ~0: finish fills them with len)
hipError_t launch_line_emit(const uint8_t* data, uint64_t len, const uint64_t* base,
                            uint64_t* start, uint64_t* end, hipStream_t s);
// rec[l].start/klen/llen; *err |= 1 if a line is 4 GiB or longer
hipError_t launch_line_finish(const uint8_t* data, uint64_t len, uint64_t nlines,
                              const uint64_t* start, const uint64_t* end, LineRec* rec,
                              uint32_t* err, hipStream_t s);
// pfx, rec[l].pfx2 / vdl, fence[j] = pfx[64 j], and the well-formed check:
// *ok &= (every line has a TAB and key[l-1] < key[l]).
hipError_t launch_line_keys(const uint8_t* data, uint64_t nlines, LineRec* rec, uint64_t* pfx,
                            uint64_t* fence, uint32_t* ok, hipStream_t s);

// dir[0 .. dir_words(nlines)) of a table whose pfx is sorted (built for every
// table; used only when the table is well-formed).
hipError_t launch_table_dir(const uint64_t* pfx, uint64_t nlines, uint32_t* dir, hipStream_t s);

// Exclusive scan of n uint64 (out[n] = total). tmp: scan_tmp_words(n) words.
uint64_t scan_tmp_words(uint64_t n);
hipError_t launch_scan_u64(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* tmp,
                           hipStream_t s);

// ---- SsTable::load's rebuild (src/sstable.rs:109-120) ----
// has[l] = line l has a TAB, klen[l] = its key length (0 without a TAB);
// *bad = min(*bad, first line whose key is not UTF-8).
hipError_t launch_rebuild_mark(const uint8_t* data, const LineRec* rec, uint64_t nlines, uint64_t* has,
                               uint64_t* klen, uint64_t* bad, hipStream_t s);
// From the exclusive scans of has / klen (n + 1 entries each): the TAB lines'
// keys as a ragged batch out/off (has_scan[n] keys, off has_scan[n] + 1
// entries) and lmap[i] = the line of key i.
hipError_t launch_rebuild_gather(const uint8_t* data, const LineRec* rec, uint64_t nlines,
                                 const uint64_t* has_scan, const uint64_t* len_scan, uint8_t* out,
                                 uint64_t* off, uint64_t* lmap, hipStream_t s);

// ---- resolution ----
// line[k] = SsTable::binary_search(key k) over one table, or -1.
hipError_t launch_table_search(int keyk, const TableView& t, const KeySrc& ks, uint64_t n,
                               int64_t* line, hipStream_t s);
// Database::get's walk over tv[0..nt) (tv[0] newest). Table t is asked only
// where hits (nullable, [rows][hwords]) has bit k of row rows[t] (rows
// nullable = identity). which[k] = first t whose line decodes as base64,
// else -1; vsrc[k] the device address of that value's base64 bytes; dlen[k]
// the decoded length (0 if none); tsum[b] = the sum of dlen over key tile b
// (kDecodeTile keys, get_tiles(n) entries).
constexpr uint32_t kDecodeTile = 256;
inline uint64_t get_tiles(uint64_t n) { return (n + kDecodeTile - 1) / kDecodeTile; }
// Database::get in one launch: the FilterSet gate (set_key_mask over the
// set of `width` slots, zones nullable) computed per key, then the same walk
// and outputs as launch_get_many; table t is slot slots[t] (nullptr: slot t),
// nt <= width.
hipError_t launch_set_get_many(int keyk, int mode, uint32_t width, const void* set, const ModP& mp,
                               const ZoneView* zones, const TableView* tv, uint32_t nt, const uint32_t* slots,
                               const KeySrc& ks, uint64_t n, int32_t* which, uint64_t* vsrc, uint64_t* dlen,
                               uint64_t* tsum, hipStream_t s);
hipError_t launch_get_many(int keyk, const TableView* tv, uint32_t nt, const uint64_t* hits,
                           const uint32_t* rows, uint64_t hwords, const KeySrc& ks, uint64_t n,
                           int32_t* which, uint64_t* vsrc, uint64_t* dlen, uint64_t* tsum,
                           hipStream_t s);
// Tile sums -> their exclusive scan in place; *total_out = the sum (one
// single-block kernel; producers leave one sum per tile, consumers read their
// block's base in one load, so no full-length scan pass).
hipError_t launch_tile_scan(uint64_t* tsum, uint64_t nt, uint64_t* total_out, hipStream_t s);
// voff[0..n) = exclusive scan of dlen from the scanned tsum (voff[n] is the
// total launch_tile_scan wrote), and the decoded values into out + voff[k];
// values are written only when out != nullptr and the total fits in cap.
hipError_t launch_b64_decode(const uint64_t* vsrc, const uint64_t* dlen, const uint64_t* tsum,
                             uint64_t n, uint64_t* voff, uint8_t* out, uint64_t cap, hipStream_t s);

}  // namespace cb
