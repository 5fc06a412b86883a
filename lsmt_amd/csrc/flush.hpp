// flush.hpp — SsTable::create's data file on the device (flush.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "sstable.hpp"

namespace cb {

// Sort record of one entry: the key's first 16 bytes as big-endian words
// (zero-padded), its length (clamped) and the entry's input index.
struct SortKey {
  uint64_t w0, w1;
  uint32_t len, idx;
};

// The first min(len, 16) bytes at src as zero-padded big-endian words, from
// the aligned dwords that contain them (a dword never crosses a page edge, so
// these loads stay inside mapped memory however src is aligned).
__device__ __forceinline__ void load16(const uint8_t* src, uint64_t len, uint64_t& w0, uint64_t& w1) {
  const uint64_t m = len < 16 ? len : 16;
  if (m == 16 && !((uintptr_t)src & 15)) {  // an aligned 16-byte key (fixed-length batches): one dwordx4
    const uint4 v = *reinterpret_cast<const uint4*>(src);
    w0 = (uint64_t)__builtin_bswap32(v.x) << 32 | __builtin_bswap32(v.y);
    w1 = (uint64_t)__builtin_bswap32(v.z) << 32 | __builtin_bswap32(v.w);
    return;
  }
  uint32_t d[5] = {0, 0, 0, 0, 0};
  const uint64_t a0 = (uint64_t)(uintptr_t)src;
  const uint32_t* base = reinterpret_cast<const uint32_t*>((uintptr_t)(a0 & ~3ull));
  const uint32_t sh = (uint32_t)(a0 & 3);
  const uint32_t nd = m ? (uint32_t)((sh + m + 3) / 4) : 0;  // dwords holding the first m bytes
#pragma unroll
  for (uint32_t j = 0; j < 5; ++j)
    if (j < nd) d[j] = base[j];
  uint32_t x[4];
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) x[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
  // little-endian bytes -> big-endian words, bytes past m cleared
  const uint64_t lo = (uint64_t)x[1] << 32 | x[0], hi = (uint64_t)x[3] << 32 | x[2];
  const uint64_t b0 = __builtin_bswap64(lo), b1 = __builtin_bswap64(hi);
  w0 = m >= 8 ? b0 : (m ? b0 & ~(~0ull >> (8 * m)) : 0);
  w1 = m >= 16 ? b1 : (m > 8 ? b1 & ~(~0ull >> (8 * (m - 8))) : 0);
}

// The sort record of entry p of a key batch (kb, ko).
__device__ __forceinline__ SortKey sort_record(const uint8_t* kb, const uint64_t* ko, uint64_t p) {
  const uint64_t o0 = ko[p], kl = ko[p + 1] - o0;
  SortKey s;
  load16(kb + o0, kl, s.w0, s.w1);
  s.len = kl > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)kl;
  s.idx = (uint32_t)p;
  return s;
}

// Line p's byte length: key, TAB, base64 of the value, newline
// (src/sstable.rs:66-70).
__host__ __device__ inline uint64_t line_len(uint64_t kl, uint64_t vl) { return kl + 1 + (vl + 2) / 3 * 4 + 1; }

// What SsTable::create leaves on the device for the host, read back in one
// copy into pinned memory once the table's work has run (cb_sstable_create
// only enqueues). Every flag starts 0 (the head up to `len` is zeroed by one
// memset), so no host-written initial values are needed.
constexpr uint32_t kZoneInline = 256;  // zone bound key bytes carried inline
struct CreateResult {
  uint32_t flags[8];          // [0] unsorted (an inversion was seen), [1] a key holds '\n' / '\t',
                              // [2] not strictly increasing, [3] the bin sort could not place every
                              // record (one bin, or a group larger than its tile: the merge sort enqueued
                              // after it runs), [4] ko[n] / vo[n] above the caller's byte bounds; [5..7] 0
  uint64_t ktot, vtot;        // ko[n], vo[n]
  uint64_t dmask[kDirPos][4]; // byte values at each position of sampled keys' 8-byte prefixes (DirMap)
  uint64_t len;               // the file's length
  uint64_t idx_min, idx_max;  // input indices of the first / last key in file order
  uint32_t zlen[2];           // their full lengths
  uint8_t zkey[2][kZoneInline];
};

// out[i] = the sort record of key i.
hipError_t launch_sort_keys(const uint8_t* kb, const uint64_t* ko, uint64_t n, SortKey* out,
                            hipStream_t s);
// Lines per tile of the file's offsets: tsum holds format_tiles(n) (>= 1)
// sums of line lengths.
constexpr uint32_t kFormatTile = 256;
inline uint64_t format_tiles(uint64_t n) { return n ? (n + kFormatTile - 1) / kFormatTile : 1; }
// r->flags[0] |= (keys not in non-decreasing order); r->ktot = ko[n],
// r->vtot = vo[n], r->flags[4] |= (ko[n] > kmax or vo[n] > vmax); r->dmask
// |= the prefix bytes of kDirSample evenly spaced keys (r's head zeroed by
// the caller); tsum = the line tiles in input order (valid if sorted).
// Launches for any n, n = 0 included.
constexpr size_t kCreateHead = 32 + 16 + kDirPos * 4 * 8;  // flags, totals, dmask: zeroed per create
hipError_t launch_sorted_check(const uint8_t* kb, const uint64_t* ko, const uint64_t* vo, uint64_t n,
                               CreateResult* r, uint64_t* tsum, uint64_t kmax, uint64_t vmax, hipStream_t s);
// tsum = the line tiles in the order of the sort records.
hipError_t launch_line_sums(const SortKey* order, const uint64_t* ko, const uint64_t* vo, uint64_t n,
                            uint64_t* tsum, hipStream_t s);
// Stable sort of the records by key, hand-written (sort.hip): LDS block
// sorts of 4096 records, then merge-path rounds. tmp: entry_sort_tmp_bytes(n)
// of scratch; in must not alias out or tmp. in == nullptr: the block sort
// builds the records from the key batch itself (no launch_sort_keys pass).
// vo != nullptr: the last launch also writes, for every output p, vsp[p] =
// {vo[idx], value length} and tsum = the line tiles in sorted order (what
// launch_line_sums would), from the records it holds in registers.
// run_if (nullable, device): every launch returns at once unless *run_if !=
// 0 (SsTable::create enqueues the sort before it knows the batch's order).
uint64_t entry_sort_tmp_bytes(uint64_t n);
hipError_t launch_entry_sort(const SortKey* in, SortKey* out, SortKey* tmp, uint64_t n, const uint8_t* kb,
                             const uint64_t* ko, hipStream_t s, const uint64_t* vo = nullptr,
                             ulonglong2* vsp = nullptr, uint64_t* tsum = nullptr, const uint32_t* run_if = nullptr);
// The same order by binning (sort.hip "bin sort"): the buckets of the
// DirMap every launch derives from r->dmask (at most bin_sort_max_bins()) as
// bins (monotone in the key), groups of ~T records sorted in LDS; out = the
// sorted records, vsp / tsum as launch_entry_sort's tail. Every launch
// returns at once when r->flags[0] is 0 (the batch is sorted). r->flags[3]
// := 1 when the bins cannot take the batch (a single bin, or a group larger
// than an LDS tile): out is then incomplete, and the caller enqueues
// launch_entry_sort after it with run_if = &r->flags[3], which redoes the
// order, vsp and tsum whole. tmp: bin_sort_tmp_bytes. Enqueued without any
// host knowledge of the batch beyond n.
uint64_t bin_sort_tmp_bytes(uint64_t n, uint32_t T);
uint32_t bin_sort_max_group();  // T at most (one LDS tile)
hipError_t launch_bin_sort(const uint8_t* kb, const uint64_t* ko, uint64_t n, uint32_t T, SortKey* out, void* tmp,
                           hipStream_t s, const uint64_t* vo, ulonglong2* vsp, uint64_t* tsum, CreateResult* r);
// The file (lines at the offsets tsum and the line lengths give, then 16
// zero bytes of slack), its
// line index without re-reading it (sstable.hpp layout: entry p is line p),
// and r's flags[1] / flags[2], len and zone bounds, in one pass (n >= 1 for
// r). bytes_bound (>= the file's length) picks the LDS stage size. The index is valid only when no key holds '\n' or '\t' (a key byte the
// reference's line split or TAB search would see): flags[1] |= 1 otherwise,
// and the caller re-indexes the file. flags[2] |= (keys not strictly
// increasing: the well-formed check).
// order / vsp (nullable): the sort's records and value spans, used only when
// r->flags[0] says the batch was unsorted (a sorted batch is formatted in
// input order). Nothing is written when r->flags[4] is set.
// vsp: entry p's {value offset, value length} in sorted order
// (launch_entry_sort's), read instead of vo[order[p].idx].
// dir (nullable, with dmap_out): the table's directory, its DirMap derived
// from r->dmask (make_dirmap(dmask, n)) and stored at dmap_out, written here
// from the lines' prefixes (what launch_table_dir would build).
// inline_scan (batches of <= kFormatInlineTiles 256-line tiles): tsum holds
// the raw tile sums and k_format scans them itself (and writes r->len), so no
// launch_tile_scan goes first: the product's 1024-entry flushes save a launch.
constexpr uint64_t kFormatInlineTiles = 64;
hipError_t launch_format(const SortKey* order, const uint8_t* kb, const uint64_t* ko,
                         const uint8_t* vb, const uint64_t* vo, const uint64_t* tsum, uint64_t n,
                         uint8_t* out, LineRec* rec, uint64_t* pfx, uint64_t* fence, uint32_t* llen,
                         CreateResult* r, uint64_t bytes_bound, hipStream_t s, const ulonglong2* vsp = nullptr,
                         uint32_t* dir = nullptr, DirMap* dmap_out = nullptr, bool inline_scan = false);

}  // namespace cb
