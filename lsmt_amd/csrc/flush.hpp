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

// What SsTable::create hands back to the host, assembled on the device so that
// each of its two host round trips is one copy into pinned memory.
constexpr uint32_t kZoneInline = 256;  // zone bound key bytes carried inline
struct CreateResult {
  uint32_t flags[4];          // [0] input sorted, [1] a key holds '\n' / '\t', [2] strictly increasing
  uint64_t ktot, vtot;        // ko[n], vo[n]
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
// r->flags[0] &= (keys already in non-decreasing order); r->ktot = ko[n],
// r->vtot = vo[n]; tsum = the line tiles in input order (valid if sorted).
// Launches for any n, n = 0 included.
hipError_t launch_sorted_check(const uint8_t* kb, const uint64_t* ko, const uint64_t* vo, uint64_t n,
                               CreateResult* r, uint64_t* tsum, hipStream_t s);
// tsum = the line tiles in the order of the sort records.
hipError_t launch_line_sums(const SortKey* order, const uint64_t* ko, const uint64_t* vo, uint64_t n,
                            uint64_t* tsum, hipStream_t s);
// Stable sort of the records by key, hand-written (sort.hip): LDS block
// sorts of 2048 records, then merge-path rounds. tmp: entry_sort_tmp_bytes(n)
// of scratch; in must not alias out or tmp.
uint64_t entry_sort_tmp_bytes(uint64_t n);
hipError_t launch_entry_sort(const SortKey* in, SortKey* out, SortKey* tmp, uint64_t n, const uint8_t* kb,
                             const uint64_t* ko, hipStream_t s);
// The same order through rocPRIM's merge sort (kept for comparison,
// CB_SORT=rocprim). tmp == nullptr: only writes the scratch size to tmp_bytes.
hipError_t entry_sort(void* tmp, size_t& tmp_bytes, const SortKey* in, SortKey* out, uint64_t n,
                      const uint8_t* kb, const uint64_t* ko, hipStream_t s);
// The file (lines at the offsets tsum and the line lengths give, then 16
// zero bytes of slack), its
// line index without re-reading it (sstable.hpp layout: entry p is line p),
// and r's flags[1] / flags[2], len and zone bounds, in one pass (n >= 1 for
// r). bytes_bound (>= the file's length) picks the LDS stage size. The index is valid only when no key holds '\n' or '\t' (a key byte the
// reference's line split or TAB search would see): flags[1] |= 1 otherwise,
// and the caller re-indexes the file. flags[2] &= (keys strictly increasing:
// the well-formed check).
hipError_t launch_format(const SortKey* order, const uint8_t* kb, const uint64_t* ko,
                         const uint8_t* vb, const uint64_t* vo, const uint64_t* tsum, uint64_t n,
                         uint8_t* out, LineRec* rec, uint64_t* pfx, uint64_t* fence, CreateResult* r,
                         uint64_t bytes_bound, hipStream_t s);

}  // namespace cb
